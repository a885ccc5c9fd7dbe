#!/bin/bash
# cfg5: level spread phase clocks, and the kernel stats of a cfg5 bench
set -o pipefail
out=gpurun_out/r03i; mkdir -p $out
tools/stamps_run.sh r03i cfg5 || exit 1
grep "spread stamps" $out/stamps_cfg5.err | tail -1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof5 -o k -- python3 bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline > $out/prof5.log 2>&1 || exit 1
find $out/prof5 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/cfg5_kernel_stats.csv
python3 - <<'P'
import csv
rows=list(csv.DictReader(open('gpurun_out/r03i/cfg5_kernel_stats.csv')))
for r in rows[:14]:
    print(r['Name'][:60].ljust(62), r['Calls'], '%.3f'%(float(r['AverageNs'])/1e6))
P
