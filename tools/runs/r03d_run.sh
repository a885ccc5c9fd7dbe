# counted-add launch under its own name; SQ counters of the sweeps on this build
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03d; mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/cfg4.json 2> $out/cfg4.err || { tail -5 $out/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/cfg4.json'));print('%.3e'%d['value'], d['breakdown_ms'], d['roofline']['kernel_ms'], d['roofline']['lds_atomic'])"
bash tools/pmc_sq.sh $out/sq || exit 1
python3 -c "
import json;d=json.load(open('$out/sq.json'))
for k,v in d.items():
    if 'sweep' in k: print(k, {c:'%.3g'%x for c,x in v.items()})"
