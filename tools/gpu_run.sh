#!/bin/bash
# GPU check used through gpurun: tests (optional), benches, optional rocprof kernel stats.
# Usage: tools/gpu_run.sh <tag> [tests] [bench:<config>[:<steps>]]... [prof:<config>]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for job in "$@"; do
  case $job in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 $out/pytest.log
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    bench:*)
      IFS=: read -r _ cfg steps <<< "$job"; steps=${steps:-5}
      timeout -k 10 400 python -u bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline > $out/bench_$cfg.json 2> $out/bench_$cfg.err
      rc=$?; echo "bench $cfg rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench_$cfg.err; exit $rc; }
      python3 -c "import json;d=json.load(open('$out/bench_$cfg.json'));print('$cfg', '%.3e'%d['value'], d['breakdown_ms'], 'frac %.3f'%d['roofline']['frac'])" ;;
    prof:*)
      cfg=${job#prof:}
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $out/prof_$cfg.log 2>&1
      rc=$?; echo "prof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
      f=$(find $out/prof_$cfg -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-160 ;;
  esac
done
