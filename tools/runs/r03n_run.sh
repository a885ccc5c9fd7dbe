# re-entry check of the restored tree: GPU tests, then per-dispatch kernel traces of cfg4/cfg5/cfg3
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03n; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in cfg4 cfg5 cfg3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/trace_$cfg -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $out/trace_$cfg.json 2> $out/trace_$cfg.err || exit 1
  echo "$cfg traced"
done
