"""Per-kernel averages of the counter passes written by profiles/run_pmc.sh."""
import collections
import csv
import glob
import json
import sys

out_dir = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for path in sorted(glob.glob(f"{out_dir}/pass*/pmc_counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
        key = (path, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
res = {}
for k in agg:
    res[k] = {c: v / cnt[k][c] for c, v in agg[k].items()}
    res[k]["avg_duration_ns"] = sum(dur[k]) / len(dur[k])
json.dump(res, sys.stdout, indent=1)
