# the shipped tree: the whole GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03y; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
tail -1 $out/smoke.log
