#!/bin/bash
# Multi-rank rehearsal of bench.py on ONE GPU: N ranks (torchrun) share cuda:0,
# gloo exchanges staged through the host.  Checks the N > 1 wiring (slab
# geometry, halo fill / ghost sum, migration, max-over-ranks timing) on the
# device path; the timings are not the metric (the driver's RCCL run is).
# Usage: tools/rehearse_multi.sh <tag> <nranks> [bench args...]
set -o pipefail
out=gpurun_out/$1; n=$2; shift 2
mkdir -p $out
export TMPDIR=/tmp IBTK_BENCH_BACKEND=gloo IBTK_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
  --master-port $((29500 + n)) bench.py --gpus $n --no-cpu-baseline "$@" > $out/rehearse_$n.json 2> $out/rehearse_$n.err \
  || { echo "rehearsal N=$n failed"; tail -20 $out/rehearse_$n.err; exit 1; }
cat $out/rehearse_$n.json
