# Round-3 end measurement of the shipped build: smoke, PMC traffic of cfg4 (copied to
# profiles/pmc_cfg4_IB_4_1gpu.json so the bench line carries it), the default bench line
# (CPU baseline included), rocprofv3 kernel stats of the same workload, the other configs,
# and a moving cfg4 step with redistribution
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03final; mkdir -p $out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
bash tools/pmc_traffic.sh $out/pmc cfg4 IB_4 > $out/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $out/pmc.log; exit 1; }
cp $out/pmc/pmc.json profiles/pmc_cfg4_IB_4_1gpu.json
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail -5 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 || { echo "prof failed"; tail -5 $out/prof.log; exit 1; }
echo "prof ok"
for cfg in cfg2 cfg3 cfg5; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { echo "$cfg failed"; tail -5 $out/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench_$cfg.json'));print('$cfg', '%.3e'%d['value'], round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['breakdown_ms'].items()}, 'frac %.3f'%d['roofline']['frac'], 'lds', d['roofline'].get('lds_atomic',{}).get('frac'))"
done
timeout -k 10 400 python -u bench.py --move --renumber --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_cfg4_move.json 2> $out/bench_cfg4_move.err || { echo "move failed"; tail -5 $out/bench_cfg4_move.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_cfg4_move.json'));print('cfg4 move+renumber', '%.3e'%d['value'], round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['breakdown_ms'].items()})"
