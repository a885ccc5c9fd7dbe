#!/bin/bash
# spread add-loop variants (IBTK_LE_DBG) with phase clocks: tools/dbg_variants.sh <tag>
out=gpurun_out/$1; mkdir -p $out
for m in ${MODES:-0 1 2 3}; do
  IBTK_LE_DBG=$m IBTK_LE_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/d$m.json 2> $out/d$m.err || exit 1
  echo "mode $m: $(grep stamps $out/d$m.err | tail -1)"
  python3 -c "import json;d=json.load(open('$out/d$m.json'));print('   spread ms', d['breakdown_ms']['spread'])"
done
