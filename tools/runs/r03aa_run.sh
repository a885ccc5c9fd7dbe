# interp ring groups of 5 anchor planes on 4 waves (ig5: 9-slot ring, 53 KB, 3 workgroups per CU): parity, cfg4/cfg5 A/B
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03aa; mkdir -p $out
IBTK_LE_LIB=$PWD/ibamr_amd/lib/var/ig5/libibtk_le.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_level.py tests/test_gpu_items.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests_ig5.log 2>&1; rc=$?
echo "ig5 tests rc=$rc"; tail -2 $out/tests_ig5.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03aa cfg4 5 3 default ig5 || exit 1
bash tools/var_ab.sh r03aa cfg5 10 1 default ig5 || exit 1
