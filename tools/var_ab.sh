#!/bin/bash
# A/B of library builds on one config, interleaved (A B A B ...) so drift hits both:
#   tools/var_ab.sh <tag> <config> <steps> <rounds> <variant>...
# <variant> is "default" (ibamr_amd/lib/libibtk_le.so) or a name built with
# IBTK_LE_VARIANT=<name> python -m ibamr_amd.build (ibamr_amd/lib/var/<name>/).
# Extra bench arguments: BENCH_ARGS="--kernel IB_6" tools/var_ab.sh ...
set -o pipefail
out=gpurun_out/$1; cfg=$2; steps=$3; rounds=$4; shift 4; mkdir -p $out
export TMPDIR=/tmp
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=ibamr_amd/lib/libibtk_le.so; else lib=ibamr_amd/lib/var/$v/libibtk_le.so; fi
    f=$out/${cfg}_${v}_$r
    IBTK_LE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline $BENCH_ARGS > $f.json 2> $f.err || { echo "$v failed"; tail -5 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f.json'));print('$cfg $v r$r', '%.3e'%d['value'], round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
  done
done
