#!/bin/bash
# XCD block dealing: GPU tests, then cfg5 / cfg4 A/B over xcd_block, cfg5 kernel stats
set -o pipefail
out=gpurun_out/r03l; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_cfg.sh r03l cfg5 5 '' '--tune xcd_block=4' '--tune xcd_block=16' '--tune xcd_block=-1' || exit 1
tools/ab_cfg.sh r03l cfg4 5 '' '--tune xcd_block=34' '--tune xcd_block=8' '--tune xcd_block=1' || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof5 -o k -- python3 bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline > $out/prof5.log 2>&1 || exit 1
f=$(find $out/prof5 -name "k_kernel_stats.csv" | head -1); cp $f $out/cfg5_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$out/cfg5_kernel_stats.csv')))[:16]: print(r['Name'][:64].ljust(66), r['Calls'], '%.3f'%(float(r['AverageNs'])/1e6))"
