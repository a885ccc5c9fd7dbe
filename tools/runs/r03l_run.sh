# interp traffic vs layout and item order: FETCH/WRITE per sweep, and timing
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03l; mkdir -p $out
i=0
for a in "" "--layout aligned" "--tune strip=2" "--layout aligned --tune strip=2"; do
  i=$((i+1))
  BENCH_ARGS="$a" bash tools/pmc_traffic.sh $out/pmc$i cfg4 IB_4 > $out/pmc$i.log 2>&1 || { tail -3 $out/pmc$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline $a > $out/b$i.json 2> $out/b$i.err || exit 1
  python3 -c "
import json;p=json.load(open('$out/pmc$i/pmc.json'));d=json.load(open('$out/b$i.json'))
print('[$a]', '%.3e'%d['value'], {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()}, {k:round(v/1e9,1) for k,v in p['per_launch_bytes'].items()}, 'read', {k:round(v/1e9,1) for k,v in p['read_bytes'].items()})"
done
