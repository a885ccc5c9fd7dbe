# key-frame components on a 5-slot spread ring: the -m gpu suite, then A/B against the previous build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03h/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03h/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03h cfg4 10 2 prev default || exit 1
bash tools/var_ab.sh r03h cfg5 10 1 prev default || exit 1
BENCH_ARGS="--kernel IB_6" bash tools/var_ab.sh r03h cfg3 5 1 prev default
