#!/bin/bash
# tools/tune_sweep.py plain + FETCH_SIZE + WRITE_SIZE passes, joined.
# Usage: tools/tune_run.sh <outdir> '<settings json>' [--config cfgN]
set -o pipefail
out=$1; st=$2; shift 2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/tune_sweep.py "$st" "$@" > $out/sweep.jsonl 2> $out/sweep.err || { echo "sweep failed"; tail -5 $out/sweep.err; exit 1; }
cat $out/sweep.jsonl | cut -c1-200
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $out/$ctr -o pmc -- python3 -u tools/tune_sweep.py "$st" "$@" > $out/$ctr.jsonl 2> $out/$ctr.err || { echo "$ctr pass failed"; tail -5 $out/$ctr.err; exit 1; }
done
python3 tools/tune_join.py $out/sweep.jsonl $out/FETCH_SIZE $out/WRITE_SIZE | tee $out/joined.jsonl
