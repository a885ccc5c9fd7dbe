#!/bin/bash
# spread ring-depth groups side by side: GPU tests, cfg4/cfg5 A/B (full ring; groups one after the other)
set -o pipefail
out=gpurun_out/r03t; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/diag_variants.sh r03t cfg4 default zfull seq default zfull || exit 1
STEPS=5 tools/diag_variants.sh r03t5 cfg5 default zfull seq || exit 1
