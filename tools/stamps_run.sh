#!/bin/bash
# Spread phase clocks and item-time spread (a -DIBTK_LE_CLOCKS=1 build in
# ibamr_amd/lib/var/clocks): tools/stamps_run.sh <tag> <config> [bench args...]
set -o pipefail
out=gpurun_out/$1; cfg=$2; shift 2; mkdir -p $out
export IBTK_LE_LIB=$PWD/ibamr_amd/lib/var/clocks/libibtk_le.so IBTK_LE_STAMPS=1
timeout -k 10 300 python -u bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline "$@" > $out/stamps_$cfg.json 2> $out/stamps_$cfg.err || { tail -5 $out/stamps_$cfg.err; exit 1; }
grep stamps $out/stamps_$cfg.err | tail -2
