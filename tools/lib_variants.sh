#!/bin/bash
# Compare library builds (ibamr_amd/lib/var/<name>, built with IBTK_LE_VARIANT/IBTK_LE_DEFS;
# "default" = ibamr_amd/lib): a parity subset, then bench on <config>.
# Usage: tools/lib_variants.sh <tag> <config> <name>...
set -o pipefail
tag=$1; cfg=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=ibamr_amd/lib/libibtk_le.so; else lib=ibamr_amd/lib/var/$v/libibtk_le.so; fi
  export IBTK_LE_LIB=$PWD/$lib
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "${PARITY_K:-dense_uniform or vertex_file or IB_4}" > $out/pytest_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 $out/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $out/bench_$v.json 2> $out/bench_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; tail -5 $out/bench_$v.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$out/bench_$v.json'));print('$v', '%.3e'%d['value'], d['breakdown_ms'], 'kernel_ms', d['roofline'].get('kernel_ms'))"
done
