#!/bin/bash
# new parity tests (3-D KAT, caller-order spread, level interp vs oracle, select_interior, sync-free step);
# spread planes 1 vs 2 ahead (+ stream-only), nontemporal plane streams; lds_atomic on cfg3/cfg5
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03h; mkdir -p $out
# (tests passed in the previous call)
true; rc=0 #  (the parity tests passed in the previous call: gpurun_out/r03h_tests_pass.log)
tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_bench.sh r03h cfg4 pf1 pf2 pf1noproc pf2noproc nt1 nt2 nt6 nt7 || exit $?
bash tools/var_bench.sh r03h cfg5 default nt1 nt7 || exit $?
for c in cfg3 cfg5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $out/$c.json 2> $out/$c.err || exit $?
  python3 -c "import json;d=json.load(open('$out/$c.json'));print('$c', '%.3e'%d['value'], d['breakdown_ms'], d['roofline']['lds_atomic'])"
done
IBTK_BENCH_BACKEND=gloo IBTK_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 \
  --config cfg2 --no-cpu-baseline --move > $out/gloo2_cfg2_move_fixed.json 2> $out/gloo2_cfg2_move_fixed.err || exit $?
python3 -c "import json;d=json.loads(open('$out/gloo2_cfg2_move_fixed.json').read().strip().splitlines()[-1]);print('gloo2 move', '%.3e'%d['value'], d['config']['migration'], d['config']['overlap_check'])"
