#!/bin/bash
# A kernel's average duration per library variant (KPAT, default k_cand_write) (rocprofv3 --kernel-trace --stats),
# cfg4 and cfg5 with moving markers (the stream rebuilt every step; the F gather in line):
#   tools/cw_prof.sh <tag> <variant>...   ("default" = ibamr_amd/lib/libibtk_le.so)
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=ibamr_amd/lib/libibtk_le.so; else lib=ibamr_amd/lib/var/$v/libibtk_le.so; fi
  for cfg in ${CFGS:-cfg4 cfg5}; do
    d=$out/${v}_$cfg
    IBTK_LE_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --config $cfg --move --steps 8 --warmup 2 --no-cpu-baseline --tune side_gather=-1 > $d.log 2>&1 || { echo "$v $cfg failed"; tail -3 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if '${KPAT:-k_cand_write}' in r['Name']:
        print('$v $cfg', r['Name'][:40], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))"
  done
done
