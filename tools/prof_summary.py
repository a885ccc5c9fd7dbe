"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) per kernel name.

Usage: python tools/prof_summary.py <run_results.db | kernel_trace.csv> [out.csv]
Columns: name, calls, avg_ms, total_ms, pct (of the traced kernel time).
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute("select name, start, end from kernels"):
            yield name, e - s
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    agg = defaultdict(lambda: [0, 0])
    for name, ns in rows_from(sys.argv[1]):
        agg[name][0] += 1
        agg[name][1] += ns
    tot = sum(v[1] for v in agg.values()) or 1
    out = [(n, c, t / c / 1e6, t / 1e6, 100.0 * t / tot) for n, (c, t) in agg.items()]
    out.sort(key=lambda r: -r[3])
    w = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["name", "calls", "avg_ms", "total_ms", "pct"])
    for r in out:
        w.writerow([r[0], r[1], f"{r[2]:.4f}", f"{r[3]:.3f}", f"{r[4]:.2f}"])


if __name__ == "__main__":
    main()
