#!/bin/bash
# plane interp: parity, then cfg4/cfg5 A/B (ring sweep vs plane sweep, VGPR budgets)
set -o pipefail
out=gpurun_out/r03a; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_cfg.sh r03a cfg4 5 '' '--tune interp_old=1' || exit 1
tools/diag_variants.sh r03a_v cfg4 ipl3 ipl5 || exit 1
tools/ab_cfg.sh r03a cfg5 5 '' '--tune interp_old=1' || exit 1
