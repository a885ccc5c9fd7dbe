#!/bin/bash
# round 3: spread planes two anchors ahead (pf2) vs the round's default and the volatile interp reads;
# moving steps with renumbering, cfg5 moving level, 2-rank gloo rehearsal of bench.py's N > 1 path
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g; mkdir -p $out
bash tools/var_bench.sh r03g cfg4 default ivol pf2 || exit $?
bash tools/var_bench.sh r03g cfg5 default pf2 || exit $?
timeout -k 10 300 python -u bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline --move --renumber \
  > $out/cfg4_move_renumber.json 2> $out/cfg4_move_renumber.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline --move \
  > $out/cfg5_move.json 2> $out/cfg5_move.err || exit $?
IBTK_BENCH_BACKEND=gloo IBTK_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  --config cfg2 --no-cpu-baseline > $out/gloo2_cfg2.json 2> $out/gloo2_cfg2.err || exit $?
IBTK_BENCH_BACKEND=gloo IBTK_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 \
  --config cfg2 --no-cpu-baseline --move --renumber > $out/gloo2_cfg2_move.json 2> $out/gloo2_cfg2_move.err || exit $?
for f in $out/*.json; do echo "$f: $(python3 -c "import json;d=json.load(open('$f'));print('%.3e'%d['value'], round(d['ms_per_step'],2), d['config'].get('overlap_check'), {k:round(v,2) for k,v in d['breakdown_ms'].items()})")"; done
