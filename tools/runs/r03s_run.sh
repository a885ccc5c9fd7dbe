# USER_DEFINED kernel function (ibtk_le_user_interp / _spread, facade form u): the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03s; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" $out/gpu_tests.log | tail -3; grep -E "FAILED|Error" $out/gpu_tests.log | head -10; exit $rc
