#!/bin/bash
# pipelined spread (variant 'pipe'): GPU tests on it, then cfg4/cfg5 A/B; interp variants ipf2/iw2
set -o pipefail
out=gpurun_out/r03e; mkdir -p $out
IBTK_LE_LIB=$PWD/ibamr_amd/lib/var/pipe/libibtk_le.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests_pipe.log 2>&1
rc=$?; tail -2 $out/tests_pipe.log; [ $rc -eq 0 ] || exit $rc
tools/diag_variants.sh r03e cfg4 pipe default ipf2 iw2 || exit 1
STEPS=5 tools/diag_variants.sh r03e5 cfg5 pipe default || exit 1
