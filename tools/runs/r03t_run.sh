# USER_DEFINED: the user-kernel tests (incl. the reference example ex4's re-scaled IB_4) and the facade
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03t; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_user.py tests/test_gpu_boundary.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" $out/gpu_tests.log | tail -2; grep -E "FAILED" $out/gpu_tests.log | head; exit $rc
