#!/bin/bash
# Round-end measurement of the default build: smoke, the default bench line (with
# the CPU baseline), rocprofv3 kernel stats of the same workload, and the
# FETCH_SIZE / WRITE_SIZE traffic passes (tools/pmc_traffic.sh).  Copy
# <out>/pmc/pmc.json to profiles/pmc_cfg4_IB_4_1gpu.json afterwards: bench.py
# reports it as roofline.traffic while its build hash matches.
# Usage: tools/final_profile.sh <tag>
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail -5 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 || { echo "prof failed"; tail -5 $out/prof.log; exit 1; }
echo "prof ok"
bash tools/pmc_traffic.sh $out/pmc cfg4 IB_4 || exit 1
echo "pmc ok"
