# interp with 8 waves per ring (iw8: 70-KB ring, 133 VGPRs; iw8h: at most 128 VGPRs, 2 workgroups
# = 16 waves per CU): interp parity on iw8h, cfg4 A/B; 2-rank rehearsal of the overlap self-check
# (now before the timed steps)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03r; mkdir -p $out
IBTK_LE_LIB=$PWD/ibamr_amd/lib/var/iw8h/libibtk_le.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_level.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests_iw8h.log 2>&1; rc=$?
echo "iw8h tests rc=$rc"; tail -2 $out/tests_iw8h.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh r03r cfg4 5 2 default iw8 iw8h || exit 1
bash tools/rehearse_multi.sh r03r 2 --steps 3 --warmup 1 || exit 1
# one GPU: ghost fill / zero beside the bin on a second stream (default) vs --serial
for r in 1 2; do for a in "" "--serial"; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline $a > $out/conc$r$a.json 2> $out/conc$r$a.err || exit 1
  python3 -c "import json;d=json.load(open('$out/conc$r$a.json'));print('conc [$a] r$r', '%.3e'%d['value'], round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['breakdown_ms'].items()})"
done; done
for a in "" "--serial"; do
  timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline $a > $out/cfg5conc$a.json 2> $out/cfg5conc$a.err || exit 1
  python3 -c "import json;d=json.load(open('$out/cfg5conc$a.json'));print('cfg5 conc [$a]', '%.3e'%d['value'], round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['breakdown_ms'].items()})"
done
