#!/bin/bash
# HBM traffic of the sweep kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE, one
# counter per pass (MI355X_MICROARCH.md, HBM section).  FETCH_SIZE is taken x2:
# on gfx950 it reports half the bytes of 8-B-per-lane reads too, not only of the
# guide's 16-B case (tools/ubench_fetch.hip + tools/calib_fetch.sh, result in
# profiles/r02b/fetch_calibration.json: k_read8 and k_read16 both 0.50);
# WRITE_SIZE is exact for contiguous stores (1.00) and counts whole 64-B pieces
# for partial ones (24-B records written 8 B at a time: 3.00).
# Writes <outdir>/pmc.json with the library's source hash; copy it to
# profiles/pmc_<cfg>_<kernel>_1gpu.json, which bench.py reads when the hash
# matches the build it runs.
# Usage: [BENCH_ARGS="..."] tools/pmc_traffic.sh <outdir> [cfg] [kernel]
# Per step: the spread sweep is one launch over all components (closed-form kernels;
# launch_spread_sweep_t); per-launch means of each kernel name are summed.
out=$1; cfg=${2:-cfg4}; kern=${3:-IB_4}
export TMPDIR=/tmp
mkdir -p "$out"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$out/$ctr" -o pmc -- \
    python3 bench.py --config $cfg --kernel $kern --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > "$out/$ctr.log" 2>&1 || { echo "$ctr pass failed"; exit 1; }
done
python3 - "$out" "$cfg" "$kern" <<'PY'
import csv, glob, json, os, sys, collections
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
sys.path.insert(0, ".")
from ibamr_amd.build import source_hash
res = {"build": source_hash(), "counters_kb": {}, "per_launch_bytes": {}, "read_bytes": {}, "write_bytes": {},
       "bench_args": os.environ.get("BENCH_ARGS", ""),
       "note": "(2 x FETCH_SIZE + WRITE_SIZE) KB x 1024 per sweep (the spread's component launches summed), mean over steps; FETCH_SIZE x 2 per "
               "profiles/r02b/fetch_calibration.json (8-B and 16-B-per-lane reads both report 0.50 of the bytes)"}
for k, d in vals.items():
    # the counted-add launch (..., true, ...>: CNT) is not the product sweep
    cnt = "k_spread_sweep" in k and k.split("<")[1].split(",")[2].strip() == "true"
    name = "spread" if "k_spread_sweep" in k and not cnt else "interp" if ("k_interp_sweep" in k or "k_interp3" in k) else None
    if name is None or not d.get("FETCH_SIZE") or not d.get("WRITE_SIZE"):
        continue
    f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
    w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    c = res["counters_kb"].setdefault(name, {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "kernels": []})
    c["FETCH_SIZE"] += f
    c["WRITE_SIZE"] += w
    c["kernels"].append(k)
for name, c in res["counters_kb"].items():
    f, w = c["FETCH_SIZE"], c["WRITE_SIZE"]
    res["per_launch_bytes"][name] = (2 * f + w) * 1024
    res["read_bytes"][name] = 2 * f * 1024
    res["write_bytes"][name] = w * 1024
json.dump(res, open(f"{out}/pmc.json", "w"), indent=1)
print(json.dumps(res))
PY
