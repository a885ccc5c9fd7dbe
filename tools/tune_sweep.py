#!/usr/bin/env python3
"""Sweep the 3-D sweeps' work-item order (ibtk_le_ctx_tune) on one resident
workload and time each setting with the library's HIP events (the context
stream).  Under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` the sweep
dispatches appear in the order printed here (REPS interp + REPS spread per
setting), so the per-dispatch counters map onto the settings.

Usage: python tools/tune_sweep.py [--config cfg4] [--reps 3] '<json list of settings>'
A setting is a dict of ctx_tune keys, e.g. {"seg_items": 16384, "split_target": 8192}.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings")
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    from ibamr_amd import le
    from ibamr_amd.slab import Slab
    cfg = bench.CONFIGS[args.config]
    kernel = args.kernel or cfg["kernel"]
    N = cfg["N"]
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    slab = Slab([N, N, N], 1, 0, g)
    geom = slab.geometry()
    dev = torch.device("cuda", 0)
    ctx = le.Context(0)
    X = bench.make_markers(cfg["markers"], cfg["M"], slab, 1234, dev)
    ci = [torch.clamp((X[:, d] / slab.dx[d]).floor().long(), 0, N - 1) for d in range(3)]
    X = X[torch.argsort((ci[2] * N + ci[1]) * N + ci[0])].contiguous()
    del ci
    M = X.shape[0]
    gen = torch.Generator(device=dev).manual_seed(4321)
    F = torch.rand((M, 3), dtype=torch.float64, device=dev, generator=gen).mul_(2).sub_(1)
    U = torch.zeros((M, 3), dtype=torch.float64, device=dev)
    u = geom.alloc("side", device=dev)
    for a in u:
        a.uniform_(-1.0, 1.0, generator=gen)
    le.fill_periodic_ghosts(ctx, geom, "side", u)
    f = geom.alloc("side", device=dev)
    bins = le.Markers(ctx)
    settings = json.loads(args.settings)
    keys = ["seg_items", "split_target", "heavy"]
    defaults = {"seg_items": 0, "split_target": 0, "heavy": 0}
    Uref = fref = None
    for i, st in enumerate(settings):
        full = dict(defaults, **st)
        for k in keys:
            ctx.tune(k, full[k])
        bins.bin(geom, kernel, X)
        ctx.enable_timing(True)
        ti, ts = [], []
        for r in range(args.reps):
            le.interp(ctx, bins, kernel, "side", geom, u, U, X)
            ctx.synchronize()
            ti.append(ctx.last_kernel_ms())
        for r in range(args.reps):
            for t in f:
                t.zero_()
            le.spread(ctx, bins, kernel, "side", geom, f, F, X)
            ctx.synchronize()
            ts.append(ctx.last_kernel_ms())
        ctx.enable_timing(False)
        # results must not depend on the order: interp bitwise, spread bitwise
        if Uref is None:
            Uref = U.clone()
            fref = [t.clone() for t in f]
            same = True
        else:
            same = bool(torch.equal(U, Uref)) and all(torch.equal(a, b) for a, b in zip(f, fref))
        print(json.dumps({"i": i, "setting": st, "interp_ms": min(ti), "spread_ms": min(ts),
                          "interp_all": ti, "spread_all": ts, "same_results": same}), flush=True)


if __name__ == "__main__":
    main()
