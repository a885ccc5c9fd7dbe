#!/bin/bash
# Bench library builds (ibamr_amd/lib/var/<name>, built with IBTK_LE_VARIANT/IBTK_LE_DEFS;
# "default" = ibamr_amd/lib) on one config, no parity run (diagnostic builds change
# results by design).  Extra env for a variant: <name>@ENV=V (e.g. clk@IBTK_LE_STAMPS=1).
# Usage: tools/var_bench.sh <tag> <config> <name>[@ENV=V]...
set -o pipefail
tag=$1; cfg=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for spec in "$@"; do
  v=${spec%%@*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*@}
  if [ "$v" = default ]; then lib=ibamr_amd/lib/libibtk_le.so; else lib=ibamr_amd/lib/var/$v/libibtk_le.so; fi
  env IBTK_LE_LIB=$PWD/$lib $envs timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-5} --warmup 2 \
      --no-cpu-baseline ${BENCH_ARGS:-} > $out/bench_${cfg}_$v.json 2> $out/bench_${cfg}_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; tail -5 $out/bench_${cfg}_$v.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$out/bench_${cfg}_$v.json'));print('$v', '%.3e'%d['value'], {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
  grep -h "stamps" $out/bench_${cfg}_$v.err | tail -2 || true
done
