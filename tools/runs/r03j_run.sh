# spread component launches side by side (default) vs one after the other (seq) vs one launch, full rings (one6)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_items.py tests/test_gpu_level.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03j/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03j/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03j cfg4 5 2 default seq one6
