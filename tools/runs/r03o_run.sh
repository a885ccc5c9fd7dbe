# cfg5 markers in the level's numbering (cell order) vs generation order; cfg4 sweep traffic
# with the items dealt round-robin over the XCDs (no L2 sharing between x-neighbour columns)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03o; mkdir -p $out
for mo in cell random; do
  timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --marker-order $mo > $out/cfg5_$mo.json 2> $out/cfg5_$mo.err || exit 1
  python3 -c "import json;d=json.load(open('$out/cfg5_$mo.json'));print('cfg5 $mo', '%.3e'%d['value'], round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['breakdown_ms'].items()}, d['roofline']['kernel_ms'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/trace_cfg5 -o run -- python3 bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $out/trace_cfg5.json 2> $out/trace_cfg5.err || exit 1
BENCH_ARGS="--tune xcd_block=1" bash tools/pmc_traffic.sh $out/pmc_rr cfg4 IB_4 > $out/pmc_rr.log 2>&1 || { tail -3 $out/pmc_rr.log; exit 1; }
bash tools/pmc_traffic.sh $out/pmc_def cfg4 IB_4 > $out/pmc_def.log 2>&1 || { tail -3 $out/pmc_def.log; exit 1; }
for v in rr def; do python3 -c "
import json;p=json.load(open('$out/pmc_$v/pmc.json'));print('$v', {k:round(v/1e9,1) for k,v in p['per_launch_bytes'].items()}, 'read', {k:round(v/1e9,1) for k,v in p['read_bytes'].items()})"; done
