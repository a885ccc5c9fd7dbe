# cfg2 (128^3 sphere, latency-bound sweeps): heavy-item split target 12288 (default) vs smaller
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03v; mkdir -p $out
for r in 1 2; do for t in 0 4096 1024 512; do
  a=""; [ $t -gt 0 ] && a="--tune split_target=$t"
  timeout -k 10 300 python -u bench.py --config cfg2 --steps 20 --warmup 3 --no-cpu-baseline $a > $out/cfg2_t${t}_${r}.json 2> $out/cfg2_t$t.err || exit 1
  python3 -c "import json;d=json.load(open('$out/cfg2_t${t}_${r}.json'));print('cfg2 split $t r$r', '%.3e'%d['value'], round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['breakdown_ms'].items()}, d['roofline']['kernel_ms'])"
done; done
