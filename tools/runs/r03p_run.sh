# spread workgroups of 2 / 4 consecutive items (IBTK_LE_SGROUP): parity subset on each variant, cfg4 A/B
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03p; mkdir -p $out
for v in sg2 sg4; do
  IBTK_LE_LIB=$PWD/ibamr_amd/lib/var/$v/libibtk_le.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_items.py tests/test_gpu_level.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -2 $out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/var_ab.sh r03p cfg4 5 2 default sg2 sg4 || exit 1
bash tools/var_ab.sh r03p cfg5 10 1 default sg2 sg4 || exit 1
