# per-dispatch traces of cfg2 and cfg5: how much of a step the GPU is busy (launch-bound or not)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03w; mkdir -p $out
for cfg in cfg2 cfg5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/trace_$cfg -o run -- python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline > $out/trace_$cfg.json 2> $out/trace_$cfg.err || exit 1
  echo "$cfg traced"
done
