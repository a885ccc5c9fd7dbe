#!/bin/bash
# cfg5 kernel stats (the one-binning step), cfg4 SQ counters of the current build
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03i; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg5 -o k -- python3 bench.py --config cfg5 \
  --steps 3 --warmup 1 --no-cpu-baseline > $out/cfg5.json 2> $out/cfg5.err || exit $?
f=$(find $out/cfg5 -name "k_kernel_stats.csv" | head -1); cp $f $out/cfg5_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$out/cfg5_kernel_stats.csv')))[:16]: print(r['Name'][:70], r['Calls'], '%.3f'%(float(r['AverageNs'])/1e6))"
bash tools/pmc_sq.sh $out/sq_cfg4 --config cfg4 || exit $?
cat $out/sq_cfg4.json | head -60
