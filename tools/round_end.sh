#!/bin/bash
# Round-end measurement set of the shipped build, one GPU call (one set, not seven):
#   the -m gpu suite, smoke(), the default bench line (with the CPU baseline), rocprofv3 kernel
#   stats of the same command, the FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh), every
#   config's line, and a 2-rank gloo rehearsal of the multi-GPU path through bench.py's own
#   launcher.  Usage: tools/round_end.sh <tag>
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail -5 $out/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_default.json'));print('default %.3e'%d['value'], round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()}, 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 || { echo "prof failed"; tail -5 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-140
bash tools/pmc_traffic.sh $out/pmc cfg4 IB_4 > $out/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $out/pmc.log; exit 1; }
python3 -c "import json;d=json.load(open('$out/pmc/pmc.json'));print('pmc', d['build'], {k:round(v/1e9,2) for k,v in d['per_launch_bytes'].items()})"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err \
    || { echo "$name failed"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', '%.3e'%d['value'], round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
}
run cfg2 --config cfg2
run cfg3_IB_6 --config cfg3 --kernel IB_6
run cfg3_BSPLINE_4 --config cfg3 --kernel BSPLINE_4
run cfg3_IB_4_W8 --config cfg3 --kernel IB_4_W8
run cfg3_IB_4 --config cfg3 --kernel IB_4
run cfg4_random --config cfg4 --marker-order random
run cfg4_move --config cfg4 --move
run cfg4_interp3 --config cfg4 --tune interp3=1
run cfg5 --config cfg5
run cfg5_move --config cfg5 --move
run cfg5_move_r10 --config cfg5 --move --regrid-every 10
IBTK_BENCH_BACKEND=gloo IBTK_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
  > $out/rehearse_2.out 2> $out/rehearse_2.err || { echo "rehearsal failed"; tail -5 $out/rehearse_2.err; exit 1; }
grep '^{' $out/rehearse_2.out > $out/rehearse_2.json
python3 -c "import json;d=json.load(open('$out/rehearse_2.json'));print('gloo rehearsal n_gpus', d['n_gpus'], d['config']['parallelism'], d['config']['overlap_check'])"
