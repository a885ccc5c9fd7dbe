#!/bin/bash
# spread ring one slot shorter for cell-frame-in-z components: GPU tests, cfg4/cfg5 A/B against the full ring
set -o pipefail
out=gpurun_out/r03s; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/diag_variants.sh r03s cfg4 default zfull default || exit 1
STEPS=5 tools/diag_variants.sh r03s5 cfg5 default zfull || exit 1
