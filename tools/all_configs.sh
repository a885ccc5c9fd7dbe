#!/bin/bash
# Bench line of every configuration (no CPU baseline): cfg2, cfg3 (IB_6, BSPLINE_4),
# cfg4 (cell order, random order, --move), cfg5.  Usage: tools/all_configs.sh <tag>
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
export TMPDIR=/tmp
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err \
    || { echo "$name failed"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/$name.json'));print('$name', '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'], d['breakdown_ms'])"
}
run cfg2 --config cfg2
run cfg3_ib6 --config cfg3 --kernel IB_6
run cfg3_bspline --config cfg3 --kernel BSPLINE_4
run cfg4 --config cfg4
run cfg4_random --config cfg4 --marker-order random
run cfg4_move --config cfg4 --move
run cfg5 --config cfg5
