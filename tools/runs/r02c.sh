set -o pipefail
out=gpurun_out/r02c; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread > $out/pytest_layout.log 2>&1; rc=$?; tail -3 $out/pytest_layout.log; [ $rc -eq 0 ] || exit $rc
for lay in aligned packed; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --layout $lay > $out/bench_$lay.json 2> $out/bench_$lay.err || { tail -5 $out/bench_$lay.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_$lay.json'));print('$lay', '%.3e'%d['value'], d['breakdown_ms'], d['roofline']['kernel_ms'])"
done
