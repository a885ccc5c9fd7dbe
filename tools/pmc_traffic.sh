#!/bin/bash
# HBM traffic of the sweep kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE, one
# counter per pass (MI355X_MICROARCH.md, HBM section).  The guide's x2 FETCH_SIZE
# correction is calibrated for 16-B-per-lane streaming reads only; the sweeps
# load 8 B per lane, and their FETCH_SIZE matches the known byte count of the
# Eulerian arrays they stream (interp: 3 x 1031 x 1030^2 x 8 B = 26.2 GB read,
# FETCH_SIZE 25.7 GB), so it is taken at face value (calibration factor 1).
# Writes <outdir>/pmc.json; copy it to profiles/pmc_<cfg>_<kernel>_1gpu.json,
# which bench.py reads.
# Usage: tools/pmc_traffic.sh <outdir> [cfg] [kernel]
out=$1; cfg=${2:-cfg4}; kern=${3:-IB_4}
export TMPDIR=/tmp
mkdir -p "$out"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$out/$ctr" -o pmc -- \
    python3 bench.py --config $cfg --kernel $kern --steps 2 --warmup 1 --no-cpu-baseline > "$out/$ctr.log" 2>&1 || { echo "$ctr pass failed"; exit 1; }
done
python3 - "$out" "$cfg" "$kern" <<'PY'
import csv, glob, json, sys, collections
out, cfg, kern = sys.argv[1:4]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for path in glob.glob(f"{out}/{ctr}/**/pmc_counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != ctr:
                continue
            per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in per.items():
            vals[k][ctr].append(v)
res = {"counters_kb": {}, "per_launch_bytes": {},
       "note": "(FETCH_SIZE + WRITE_SIZE) KB x 1024 per launch, mean over launches; FETCH_SIZE calibration factor 1 "
               "for the sweeps' 8-B-per-lane loads (see tools/pmc_traffic.sh)"}
for k, d in vals.items():
    name = "spread" if "k_spread_sweep" in k else "interp" if "k_interp_sweep" in k else None
    if name is None or not d.get("FETCH_SIZE") or not d.get("WRITE_SIZE"):
        continue
    f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
    w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    res["counters_kb"][name] = {"FETCH_SIZE": f, "WRITE_SIZE": w}
    res["per_launch_bytes"][name] = (f + w) * 1024
json.dump(res, open(f"{out}/pmc.json", "w"), indent=1)
print(json.dumps(res))
PY
