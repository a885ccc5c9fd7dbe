#!/bin/bash
# Interp / spread traffic (FETCH_SIZE, WRITE_SIZE passes) and step time for item-order settings:
#   tools/strip_pmc.sh <tag> "<tune args>"...   e.g. "" "--tune strip=2" "--tune strip=2 --tune xcd_block=16"
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  BENCH_ARGS="$a" bash tools/pmc_traffic.sh $out/pmc$i cfg4 IB_4 > $out/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $out/pmc$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $a > $out/b$i.json 2> $out/b$i.err || { echo "bench $i failed"; exit 1; }
  python3 -c "
import json
p=json.load(open('$out/pmc$i/pmc.json')); d=json.load(open('$out/b$i.json'))
print(repr('$a'), 'interp %.1f GB (r %.1f w %.1f)' % (p['per_launch_bytes']['interp']/1e9, p['read_bytes']['interp']/1e9, p['write_bytes']['interp']/1e9), 'spread %.1f GB' % (p['per_launch_bytes']['spread']/1e9), '%.3e' % d['value'], {k: round(v, 2) for k, v in d['roofline']['kernel_ms'].items()})"
done
