#!/bin/bash
# A/B of bench.py argument sets on one config: tools/ab_cfg.sh <tag> <config> <steps> '<args A>' '<args B>' ...
set -o pipefail
out=gpurun_out/$1; cfg=$2; steps=$3; shift 3; mkdir -p $out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline $a > $out/ab_${cfg}_$i.json 2> $out/ab_${cfg}_$i.err || { tail -5 $out/ab_${cfg}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/ab_${cfg}_$i.json'));print('$cfg [$a]', '%.3e'%d['value'], {k:round(v,2) for k,v in d['breakdown_ms'].items()}, 'kernel_ms', {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
done
