#!/bin/bash
# SQ/LDS counters of the sweep kernels over tools/tune_sweep.py (one setting),
# one counter group per rocprofv3 pass (<= 8 SQ counters each).
# Usage: tools/sq_run.sh <outdir> ['<settings json>'] [tune_sweep args...]
set -o pipefail
out=$1; st=${2:-'[{}]'}; shift 2
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/g$i -o pmc -- python3 -u tools/tune_sweep.py "$st" "$@" > $out/g$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/g$i.log; exit 1; }
done
python3 - $out <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(f"{out}/g*/**/pmc_counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "k_interp_sweep" not in k and "k_spread_sweep" not in k:
            continue
        kk = "interp" if "k_interp_sweep" in k else "spread"
        per[(kk, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (kk, d, c), v in per.items():
        acc[kk][c].append(v)
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
json.dump(res, open(f"{out}/sq.json", "w"), indent=1)
for k, d in res.items():
    wc = d.get("SQ_WAVE_CYCLES", 1)
    print(k, {c: round(v / 1e6, 1) for c, v in sorted(d.items())})
    if "SQ_LDS_IDX_ACTIVE" in d:
        print("  lds conflict share %.2f" % (d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1)))
    print("  wait_any %.2f wait_inst %.2f active %.2f of wave cycles" % (d.get("SQ_WAIT_ANY", 0) / wc, d.get("SQ_WAIT_INST_ANY", 0) / wc, d.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
