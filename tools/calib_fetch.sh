#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/ubench_fetch.hip),
# one counter group per rocprofv3 pass, no tracing besides the kernel trace.
# Usage: tools/calib_fetch.sh <outdir>
set -o pipefail
out=$1; mkdir -p $out
export TMPDIR=/tmp
./tools/ubench_fetch > $out/bytes.json || exit 1
for grp in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/$tag -o pmc -- ./tools/ubench_fetch > $out/$tag.log 2>&1 || { echo "pass $grp failed"; tail -3 $out/$tag.log; }
done
python3 - $out <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
nb = json.load(open(f"{out}/bytes.json"))
res = collections.defaultdict(dict)
for path in glob.glob(f"{out}/**/pmc_counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        per[(r["Kernel_Name"].split("(")[0].split()[-1], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    agg = collections.defaultdict(list)
    for (k, d, c), v in per.items():
        agg[(k, c)].append(v)
    for (k, c), v in agg.items():
        res[k][c] = sum(v) / len(v)
summ = {}
for k, d in res.items():
    b = nb.get(k)
    if not b:
        continue
    e = {"bytes": b}
    if "FETCH_SIZE" in d: e["FETCH_SIZE_bytes/true"] = d["FETCH_SIZE"] * 1024 / b
    if "WRITE_SIZE" in d: e["WRITE_SIZE_bytes/true"] = d["WRITE_SIZE"] * 1024 / b
    for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"):
        if c in d: e[c + "_per_128B"] = d[c] * 128 / b
    summ[k] = e
json.dump(summ, open(f"{out}/calib.json", "w"), indent=1)
print(json.dumps(summ, indent=1))
PY
