#!/bin/bash
# A/B of one tuning key on one config, interleaved (A B A B ...) so drift hits both:
#   tools/tune_ab.sh <tag> <rounds> <key> <valueA> <valueB> <bench args...>
set -o pipefail
out=gpurun_out/$1; rounds=$2; key=$3; va=$4; vb=$5; shift 5; mkdir -p $out
export TMPDIR=/tmp
for r in $(seq 1 $rounds); do
  for v in $va $vb; do
    f=$out/${key}_${v}_$r
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --tune $key=$v "$@" > $f.json 2> $f.err || { echo "$key=$v failed"; tail -5 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f.json'));print('$key=$v r$r', '%.3e'%d['value'], round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
  done
done
