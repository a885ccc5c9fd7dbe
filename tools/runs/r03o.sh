#!/bin/bash
# every config's bench line, then the multi-rank rehearsal (N=2, N=2 --move, N=4) on one GPU
set -o pipefail
tools/all_configs.sh r03o || exit 1
tools/rehearse_multi.sh r03o 2 --steps 3 --warmup 1 > /dev/null || exit 1
tools/rehearse_multi.sh r03o_m 2 --steps 3 --warmup 1 --move > /dev/null || exit 1
tools/rehearse_multi.sh r03o 4 --steps 3 --warmup 1 --spread-mode markers > /dev/null || exit 1
for f in gpurun_out/r03o/rehearse_2.json gpurun_out/r03o_m/rehearse_2.json gpurun_out/r03o/rehearse_4.json; do
  python3 -c "import json;d=json.load(open('$f'));print('$f', '%.3e'%d['value'], d['n_gpus'], d.get('breakdown_ms'))"
done
