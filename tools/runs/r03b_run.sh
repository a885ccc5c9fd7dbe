set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not split and not rank" > gpurun_out/r03b/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03b/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03b cfg4 10 2 base default
