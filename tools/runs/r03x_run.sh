# heavy spread items on HPARTS waves (HV launch on a second stream): GPU tests, cfg5/cfg2/cfg4 A/B vs the previous build
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03x; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -2 $out/gpu_tests.log; grep -E "FAILED" $out/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03x cfg5 10 2 prev default || exit 1
bash tools/var_ab.sh r03x cfg2 20 2 prev default || exit 1
bash tools/var_ab.sh r03x cfg4 5 1 prev default || exit 1
