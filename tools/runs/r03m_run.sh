# short sweep segments on narrow patches (cfg2): parity tests, cfg2 A/B, cfg4 unchanged
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03m/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03m/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03m cfg2 20 2 prev default || exit 1
bash tools/var_ab.sh r03m cfg4 5 1 prev default
