#!/bin/bash
set -o pipefail
out=gpurun_out/r03y; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_cfg.sh r03y cfg5 10 '' || exit 1
tools/final_profile.sh r02final6
