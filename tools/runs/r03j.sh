#!/bin/bash
# the whole -m gpu suite on this build, then cfg5 / cfg4 bench lines
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03j; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for c in cfg5 cfg4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $out/$c.json 2> $out/$c.err || exit $?
  python3 -c "import json;d=json.load(open('$out/$c.json'));print('$c', '%.3e'%d['value'], round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['breakdown_ms'].items()}, d['roofline']['kernel_ms'])"
done
