#!/bin/bash
# direct-F spread candidates (no gather pass): parity subset, then cfg4 (cell and random marker order) and cfg5
set -o pipefail
tools/lib_variants.sh r03d cfg4 fdirect default || exit 1
STEPS=5 tools/diag_variants.sh r03d5 cfg5 fdirect default || exit 1
for v in fdirect default; do
  if [ $v = default ]; then lib=ibamr_amd/lib/libibtk_le.so; else lib=ibamr_amd/lib/var/$v/libibtk_le.so; fi
  IBTK_LE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline --marker-order random > gpurun_out/r03d/rand_$v.json 2>gpurun_out/r03d/rand_$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r03d/rand_$v.json'));print('random $v', '%.3e'%d['value'], {k:round(v,2) for k,v in d['breakdown_ms'].items()}, d['roofline']['kernel_ms'])"
done
