# XCD block size of the sweep item dealing (ctx_tune xcd_block; default 8 table entries)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03z; mkdir -p $out
for r in 1 2; do for b in 8 4 16 32; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --tune xcd_block=$b > $out/cfg4_b${b}_${r}.json 2> $out/cfg4_b${b}.err || exit 1
  python3 -c "import json;d=json.load(open('$out/cfg4_b${b}_${r}.json'));print('cfg4 xcd_block $b r$r', '%.3e'%d['value'], round(d['ms_per_step'],2), d['roofline']['kernel_ms'])"
done; done
