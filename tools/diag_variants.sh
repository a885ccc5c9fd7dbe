#!/bin/bash
# Bench-only comparison of diagnostic library builds (no parity: the variants
# change results by design).  tools/diag_variants.sh <tag> <config> <name>...
set -o pipefail
tag=$1; cfg=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for v in "$@"; do
  if [ "$v" = default ]; then lib=ibamr_amd/lib/libibtk_le.so; else lib=ibamr_amd/lib/var/$v/libibtk_le.so; fi
  IBTK_LE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $out/bench_$v.json 2> $out/bench_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; tail -5 $out/bench_$v.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$out/bench_$v.json'));print('$v', '%.3e'%d['value'], {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
done
