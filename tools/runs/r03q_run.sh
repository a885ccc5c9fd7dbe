# bucket starts by a suffix-min scan, interp split by z frame (key-frame ring 40 KB, 16 waves per CU):
# XCD-contiguous gathers (gxcd0 = off); full GPU tests, cfg4/cfg5 A/B against the previous build, cfg3 SQ counters (IB_6 spread bank conflicts)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03q; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03q cfg4 5 2 prev default iwpe1 gxcd0 || exit 1
bash tools/var_ab.sh r03q cfg5 10 1 prev default gxcd0 || exit 1
bash tools/pmc_sq.sh $out/sq_cfg3 --config cfg3 > $out/sq_cfg3.log 2>&1 || { tail -3 $out/sq_cfg3.log; exit 1; }
echo sq done
