#!/bin/bash
# ghost passes 4 points a thread along dim 0: GPU tests, cfg4 bench
set -o pipefail
out=gpurun_out/r03p; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_cfg.sh r03p cfg4 10 '' || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o k -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
f=$(find $out/prof -name "k_kernel_stats.csv" | head -1); cp $f $out/cfg4_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$out/cfg4_kernel_stats.csv')))[:10]: print(r['Name'][:64].ljust(66), r['Calls'], '%.3f'%(float(r['AverageNs'])/1e6))"
