#!/usr/bin/env python3
"""Join rocprofv3 PMC passes of tools/tune_sweep.py with its settings (dispatch
order: per setting REPS interp sweeps then REPS spread sweeps).  FETCH_SIZE is
taken x2 and WRITE_SIZE x1 (tools/ubench_fetch.hip calibration, profiles/r02/calib.json).
Usage: tune_join.py <sweep stdout> <pmc dir>... """
import collections, csv, glob, json, sys

lines = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
reps = len(lines[0]["interp_all"])
vals = {}
for d in sys.argv[2:]:
    for path in glob.glob(f"{d}/**/pmc_counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if "k_interp_sweep" not in k and "k_spread_sweep" not in k:
                continue
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = "interp" if "k_interp_sweep" in k else "spread"
        for (disp, ctr), v in per.items():
            vals.setdefault(ctr, {})[disp] = (names[disp], v)
out = []
for ctr, dd in vals.items():
    seq = [dd[k] for k in sorted(dd)]
    fac = 2048.0 if ctr == "FETCH_SIZE" else 1024.0
    for i, l in enumerate(lines):
        chunk = seq[i * 2 * reps:(i + 1) * 2 * reps]
        for kind in ("interp", "spread"):
            v = [x for n, x in chunk if n == kind]
            if v:
                l.setdefault("bytes", {})[f"{kind}_{ctr}"] = sum(v) / len(v) * fac
for l in lines:
    print(json.dumps({k: l[k] for k in ("i", "setting", "interp_ms", "spread_ms", "same_results", "bytes") if k in l}))
