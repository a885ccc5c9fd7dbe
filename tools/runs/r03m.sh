#!/bin/bash
# block dealing default 8, level fill with a neighbour table: GPU tests, cfg5 and cfg4 benches
set -o pipefail
out=gpurun_out/r03m; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_cfg.sh r03m cfg5 10 '' || exit 1
tools/ab_cfg.sh r03m cfg4 10 '' || exit 1
