"""One step's kernel dispatches from a rocprofv3 kernel_trace.csv.

Usage: python tools/step_kernels.py <run_kernel_trace.csv> [anchor-substring] [k]
Prints the dispatches between the k-th and (k+1)-th dispatch whose name contains the
anchor (default: the interp sweep), with durations and the gaps between them.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_interp_sweep"
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(path))), key=lambda t: t[0])
    hits = [i for i, r in enumerate(rows) if anchor in r[2]]
    a, b = hits[k], hits[k + 1]
    t0 = rows[a][0]
    tot = 0
    prev_end = None
    for s, e, n in rows[a:b]:
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        tot += e - s
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {n[:110]}")
        prev_end = e
    print(f"kernels {tot / 1e6:.3f} ms, wall {(rows[b][0] - t0) / 1e6:.3f} ms, {b - a} dispatches")


if __name__ == "__main__":
    main()
