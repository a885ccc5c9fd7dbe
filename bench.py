#!/usr/bin/env python3
"""Benchmark of the LE coupling hot path: IB_4 3-D staggered interpolate + spread.

One step = one IB coupling pass over the resident markers of every rank:
  bin      re-bin the markers by stencil anchor (device radix sort)
  fill     ghost fill of u (x/y periodic locally, z from the slab neighbours)
  interp   U = J u   (LEInteractor::interpolate, side-centred, all 3 components)
  spread   f = S F   (LDataManager::spread: f zeroed, ghosts included, then
           LEInteractor::spread into the ghosted slab -- one sweep that writes f and
           never reads it; --spread-into existing: f += S F with only the ghosts zeroed)
  sum      ghost-region sum of f (z over RCCL, x/y periodic locally)
Marker-ops per step = 2 x markers (one interpolate and one spread per marker).

Default workload = BASELINE.json configs[3] (cfg4): 1024^3 periodic staggered grid,
1e8 uniformly scattered markers (seed 1234), IB_4, fp64.  It is the configuration
the north-star target (>=1e10 marker-ops/s at >=50 % HBM roofline on one MI355X,
>=6x at 8 GPUs) is quoted on, and it fits one GPU (~62 GB).  With --gpus N the same
global problem is z-slab decomposed over N ranks (strong scaling).  --config cfg2/cfg3/
cfg5 select the other BASELINE configs.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "IB_4 3D spread+interp marker-ops/sec (fp64) + % HBM roofline, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    "cfg2": dict(N=128, M=100_000, kernel="IB_4", markers="sphere",
                 desc="cfg2: 128^3 periodic staggered grid, 1e5 markers on a sphere (r=0.35), IB_4"),
    "cfg3": dict(N=512, M=10_000_000, kernel="IB_6", markers="uniform",
                 desc="cfg3: 512^3 periodic staggered grid, 1e7 uniform markers, IB_6"),
    "cfg4": dict(N=1024, M=100_000_000, kernel="IB_4", markers="uniform",
                 desc="cfg4: 1024^3 periodic staggered grid, 1e8 uniform markers (seed 1234), IB_4, z-slabs"),
    "cfg5": dict(N=512, M=10_000_000, kernel="IB_4", markers="clustered", patches=8,
                 desc="cfg5: 512^3 multi-patch finest level (8^3 patches of 64^3), 1e7 markers in ~2% of cells "
                      "(4 sheets + 2 bundles), IB_4"),
}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_markers(kind, M, slab, seed, device):
    """Markers of this rank: those whose z lies in the rank's slab [z0, z1)*dz."""
    import torch
    g = torch.Generator(device=device).manual_seed(seed + 7919 * slab.rank)
    z_lo, z_hi = slab.z0 * slab.dx[2], slab.z1 * slab.dx[2]
    if kind == "uniform":
        m = M // slab.P + (1 if slab.rank < M % slab.P else 0)
        X = torch.rand((m, 3), dtype=torch.float64, device=device, generator=g)
        X[:, 2].mul_(z_hi - z_lo).add_(z_lo)
        return X
    if kind == "sphere":
        # Fibonacci lattice on a sphere of radius 0.35 centred at 0.5
        i = torch.arange(M, dtype=torch.float64, device=device) + 0.5
        phi = torch.acos(1 - 2 * i / M)
        theta = math.pi * (1 + 5 ** 0.5) * i
        X = torch.stack([0.5 + 0.35 * torch.cos(theta) * torch.sin(phi),
                         0.5 + 0.35 * torch.sin(theta) * torch.sin(phi),
                         0.5 + 0.35 * torch.cos(phi)], dim=1)
    elif kind == "clustered":
        # 4 thin sheets (1 cell thick) + 2 fibre bundles, ~2% of cells
        n_sheet = int(M * 0.8) // 4
        n_fib = (M - 4 * n_sheet) // 2
        h = 1.0 / slab.N[0]
        parts = []
        for k, z in enumerate((0.2, 0.4, 0.6, 0.8)):
            s = torch.rand((n_sheet, 3), dtype=torch.float64, device=device, generator=g)
            s[:, 2] = z + (s[:, 2] - 0.5) * h
            parts.append(s)
        for k, (cx, cy) in enumerate(((0.3, 0.3), (0.7, 0.6))):
            f = torch.rand((n_fib, 3), dtype=torch.float64, device=device, generator=g)
            r = 0.02 * torch.sqrt(f[:, 0])
            t = 2 * math.pi * f[:, 1]
            f[:, 0] = cx + r * torch.cos(t)
            f[:, 1] = cy + r * torch.sin(t)
            parts.append(f)
        X = torch.cat(parts)
    else:
        raise ValueError(kind)
    keep = (X[:, 2] >= z_lo) & (X[:, 2] < z_hi)
    return X[keep].contiguous()


def physical_cores(cpus):
    """The physical cores among the logical CPUs `cpus` (SMT siblings counted once), from
    /sys/devices/system/cpu/cpu*/topology; len(cpus) where the topology is unreadable."""
    cores = set()
    for c in cpus:
        t = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
        try:
            cores.add((int((t / "physical_package_id").read_text()), int((t / "core_id").read_text())))
        except (OSError, ValueError):
            return len(cpus)
    return len(cores) or len(cpus)


def cpu_quota():
    """The CPUs' worth of time this process's cgroup may use (cpu.max / cfs_quota), or None if
    unlimited or unreadable: on the GPU pool the affinity set shows the whole host (256 CPUs)
    while the quota is one GPU's share."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(cfg, kernel, seconds_target=15.0):
    """The oracle (the C restatement) timed on a bounded, same-density sample: on 1 thread, and
    on one thread per physical core of this process's affinity set (every core
    of the GPU host), one replica of the sample each, as MPI ranks each holding a patch.  The
    pool's OMP_NUM_THREADS cap (one GPU's share of a shared host) does not limit it; the record
    states the cap and also the rate at that many threads (`value_pool_share`).

    Why a sample and not cfg4 itself: the oracle's cost is per marker (a W^3 stencil each way),
    independent of the grid size, and the full problem (1e8 markers, 52 GB of u and f) would take
    minutes of CPU time and tens of GB of host memory per replica inside a bench that must
    finish in a few minutes.  Sample: a periodic N_s^3 grid with the workload's marker density
    (cell-sorted order, as on the GPU), IB_4 side-centred interp + spread (periodic images in the
    spread list, LIndexSetData semantics), repeated until ~seconds_target of CPU work.  u is
    shared read-only by the threads; f and U are per thread.
    """
    import numpy as np
    from oracle import oracle as ora
    N = cfg["N"]
    density = cfg["M"] / float(N ** 3)
    Ns = min(N, 128)
    Ms = max(1000, int(round(density * Ns ** 3)))
    if cfg["markers"] == "sphere":
        Ns, Ms = N, cfg["M"]
    rng = np.random.default_rng(1234)
    X = rng.uniform(0.0, 1.0, (Ms, 3))
    if cfg["markers"] == "sphere":
        i = np.arange(Ms) + 0.5
        phi = np.arccos(1 - 2 * i / Ms)
        th = math.pi * (1 + 5 ** 0.5) * i
        X = np.stack([0.5 + 0.35 * np.cos(th) * np.sin(phi), 0.5 + 0.35 * np.sin(th) * np.sin(phi),
                      0.5 + 0.35 * np.cos(phi)], 1)
    c = np.floor(X * Ns).astype(np.int64)
    X = X[np.lexsort((c[:, 0], c[:, 1], c[:, 2]))].copy()
    F = rng.uniform(-1, 1, (Ms, 3))
    g = ora.min_ghost_width(kernel)
    lo, hi, dx = [0, 0, 0], [Ns - 1] * 3, [1.0 / Ns] * 3
    u = [rng.uniform(-1, 1, ora.ghost_shape(*ora.side_box(lo, hi, a), [g] * 3)) for a in range(3)]
    f = [np.zeros_like(a) for a in u]
    idx_i = np.arange(Ms, dtype=np.int32)
    xs_i = np.zeros((Ms, 3))
    idx_s, xs_s, _ = ora.periodic_index_list(X, [0, 0, 0], [1, 1, 1], dx, lo, hi, g)
    def one_pass(uu, ff, UU):
        ora.side_interp(kernel, dx, [0, 0, 0], lo, hi, [g] * 3, uu, idx_i, xs_i, X, UU)
        ora.side_spread(kernel, dx, [0, 0, 0], lo, hi, [g] * 3, ff, idx_s, xs_s, X, F)

    # one thread
    U = np.zeros((Ms, 3))
    reps, elapsed = 0, 0.0
    t_one = 0.4 * seconds_target
    while elapsed < t_one or reps < 2:
        t0 = time.perf_counter()
        one_pass(u, f, U)
        elapsed += time.perf_counter() - t0
        reps += 1
        if reps >= 50:
            break
    rate1 = 2.0 * Ms * reps / elapsed
    # T threads, one replica of the sample each (as MPI ranks each holding a patch,
    # SURVEY.md 8(d)); ctypes releases the GIL inside the C calls
    import threading
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    phys_aff = physical_cores(cpus)
    quota = cpu_quota()
    # one thread per physical core the process can run on: the affinity set's, unless the cgroup's
    # CPU quota allows fewer (then more threads only time-slice the same quota)
    phys = min(phys_aff, quota) if quota else phys_aff
    cap = os.environ.get("OMP_NUM_THREADS")

    def run_threads(T, t_run):
        reps_t = [0] * T
        start = threading.Barrier(T + 1)

        def worker(k):
            ff = [np.zeros_like(a) for a in u]
            UU = np.zeros((Ms, 3))
            start.wait()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < t_run or reps_t[k] < 1:
                one_pass(u, ff, UU)
                reps_t[k] += 1

        threads = [threading.Thread(target=worker, args=(k,)) for k in range(T)]
        for th in threads:
            th.start()
        start.wait()
        t0 = time.perf_counter()
        for th in threads:
            th.join()
        wall = time.perf_counter() - t0
        return 2.0 * Ms * sum(reps_t) / wall, sum(reps_t), wall

    rateT, passes, wall = run_threads(phys, 0.3 * seconds_target)
    # beside it, fewer threads: the pool's share of the host (OMP_NUM_THREADS: one GPU's 16 of a
    # host shared by 8) and the powers of two up to the physical cores -- on a shared host the
    # replicas' f arrays contend for memory bandwidth, and fewer threads may do more
    by_threads = {phys: rateT}
    share = None
    tries = {16, 32, 64, phys_aff}
    if cap and cap.isdigit() and 0 < int(cap) < phys_aff:
        tries.add(int(cap))
    for T in sorted(t for t in tries if 1 < t <= phys_aff and t != phys):
        by_threads[T] = run_threads(T, 0.1 * seconds_target)[0]
    if cap and cap.isdigit():
        share = by_threads.get(int(cap))
    best_t = max(by_threads, key=by_threads.get)
    return {"value": rateT, "unit": "marker-ops/s", "cores": phys, "kind": "port", "value_1thread": rate1,
            "value_pool_share": share, "pool_share_threads": int(cap) if share is not None else None,
            "value_by_threads": {str(k): v for k, v in sorted(by_threads.items())},
            "value_best": by_threads[best_t], "best_threads": best_t,
            "host_nproc": os.cpu_count(), "affinity_cpus": len(cpus), "physical_cores_affinity": phys_aff,
            "cgroup_cpu_quota": quota, "physical_cores": phys, "omp_num_threads": cap,
            "sample": f"{Ns}^3 periodic grid, {Ms} uniform markers (same density as the workload), "
                      f"{kernel} side interp+spread, cell-sorted (oracle C); {phys} threads (one per physical "
                      f"core of the affinity set ({phys_aff}) within the cgroup CPU quota ({quota}), "
                      f"OMP_NUM_THREADS={cap} not applied), one replica of the sample "
                      f"each: {passes} passes in {wall:.1f} s; 1 thread: {reps} passes in {elapsed:.1f} s; a "
                      f"sample, not cfg4 itself: the oracle's cost is per marker, independent of the grid"}


def level_lists(X, N, P, g):
    """LIndexSetData's per-patch lists on a level of P^3 equal patches tiling a
    periodic [0,1)^3 in torch ops -- the check for ibtk_le_level_index_lists, which the
    bench uses (tests/test_gpu_level_lists.py): the interior lists (markers whose cell is
    in the patch box, for interp) and the ghost-box lists (the markers and their
    periodic images whose cell is in the patch's ghost box, for spread,
    LDataManager.cpp:634-654).  Returns flat (indices, Xshift, offsets) per kind,
    patch-major; within a patch in marker order."""
    import torch
    n = N // P
    c = torch.clamp((X * N).floor().long(), 0, N - 1)
    t = c // n
    pid = (t[:, 2] * P + t[:, 1]) * P + t[:, 0]
    o = torch.argsort(pid, stable=True)
    cnt = torch.bincount(pid, minlength=P ** 3)
    off_i = [0] + torch.cumsum(cnt, 0).tolist()
    interior = o.to(torch.int32)
    ent_p, ent_s, ent_x = [], [], []
    ar = torch.arange(X.shape[0], device=X.device)
    for oz in (-1, 0, 1):
        for oy in (-1, 0, 1):
            for ox in (-1, 0, 1):
                off = torch.tensor([ox, oy, oz], device=X.device)
                tt = t + off                       # the tile whose ghost box may hold the cell
                shift = torch.zeros_like(tt)
                shift[tt < 0] = 1                  # tile -1 is tile P-1: the image X + L
                shift[tt >= P] = -1                # tile P is tile 0: the image X - L
                cimg = c + shift * N
                tw = tt % P
                ok = ((cimg >= tw * n - g) & (cimg <= tw * n + n - 1 + g)).all(dim=1)
                sel = ar[ok]
                ent_p.append(((tw[ok, 2] * P + tw[ok, 1]) * P + tw[ok, 0]))
                ent_s.append(sel)
                ent_x.append(shift[ok].to(torch.float64))
    ep, es, ex = torch.cat(ent_p), torch.cat(ent_s), torch.cat(ent_x)
    o2 = torch.argsort(ep * X.shape[0] + es)
    cnt2 = torch.bincount(ep, minlength=P ** 3)
    off_s = [0] + torch.cumsum(cnt2, 0).tolist()
    return (interior, None, off_i), (es[o2].to(torch.int32).contiguous(), ex[o2].contiguous(), off_s)


def binning_label(counts, full_name):
    """What the timed steps' binning did: full binnings and re-binnings, counted."""
    f, r = counts.get("full", 0), counts.get("rebin", 0)
    parts = []
    if f:
        parts.append(f"{f} full binning(s) (device radix sort, {full_name})")
    if r:
        parts.append(f"{r} re-binning(s) from the previous order (ibtk_le_markers_rebin: every key recomputed "
                     "from the current positions, the entries whose bucket changed inserted; equal to a full binning)")
    return " + ".join(parts) + " over the timed steps" if parts else "none in the timed steps (binned once at setup)"


# the reach of a kernel's stencil beyond its marker's cell (W / 2): the lists' drift slack is
# the ghost width less it
KERNEL_HALF_WIDTH = {"PIECEWISE_CONSTANT": 1, "DISCONTINUOUS_LINEAR": 1, "PIECEWISE_LINEAR": 1, "PIECEWISE_CUBIC": 2,
                     "IB_3": 2, "IB_4": 2, "IB_4_W8": 4, "IB_6": 3, "BSPLINE_4": 2}


# ds_add_f64 cost, conflict-free (tools/ubench_lds2.hip): 10 cycles
# per wave-instruction per CU at 2.4 GHz (MI355X_MICROARCH.md), 256 CUs
LDS_ADD_CYCLES, CLOCK_GHZ, NCU = 10.0, 2.4, 256


def lds_atomic(ctx, spread_call, k_ms):
    """The spread sweep's LDS-atomic bound: its ds_add_f64 counted on one extra call
    (ibtk_le_ctx_count_adds), priced at the measured conflict-free rate."""
    ctx.count_adds(True)
    spread_call()
    ctx.synchronize()
    ctx.count_adds(False)
    ins, lanes = ctx.last_adds()
    floor_ms = ins * LDS_ADD_CYCLES / (NCU * CLOCK_GHZ * 1e9) * 1e3
    return {"bound": "lds_atomic", "ds_add_wave_instr": ins, "lane_adds": lanes,
            "lane_fill": lanes / max(64 * ins, 1), "cycles_per_instr": LDS_ADD_CYCLES, "cus": NCU,
            "clock_ghz": CLOCK_GHZ, "floor_ms": floor_ms, "kernel_ms": k_ms, "frac": floor_ms / k_ms if k_ms else None,
            "note": "floor = wave-instructions x 10 cycles / (256 CUs x 2.4 GHz): the adds alone at the "
                    "conflict-free ds_add_f64 rate of tools/ubench_lds2.hip"}


# what kernel_ms times (HIP events around the sweep launches on the context stream)
KERNEL_NOTE = ("interp = k_interp_sweep<K, LVL>; spread = k_spread_sweep<K, LVL, false, ZC> over all three "
               "components in one launch (closed-form kernels: ZC, the 5-slot ring, the z-side component through "
               "the candidate stream's shifted-z split); the candidate stream's build (k_cand_count / k_cand_write, "
               "skipped on the device when the re-binning changed nothing) is outside these events")


def run_level(args, cfg, kernel, dev):
    """--config cfg5 (default): the clustered markers on a multi-patch finest level,
    8^3 patches of 64^3, one launch per sweep over every patch.
    One step = level ghost fill of u, one bin of the ghost-box lists (the interior
    lists select their entries for interp), interp, zero f, spread (the patches'
    interiors are complete: no reduction)."""
    import torch
    from ibamr_amd import le
    N, P = cfg["N"], cfg.get("patches", 8)
    n = N // P
    ctx = le.Context(dev.index or 0)
    for kv in args.tune:
        ctx.tune(kv.split("=")[0], int(kv.split("=")[1]))
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    dx = 1.0 / N
    geoms = []
    for k in range(P):
        for j in range(P):
            for i in range(P):
                lo = [i * n, j * n, k * n]
                geoms.append(le.Geometry(lo, [v + n - 1 for v in lo], g, [dx] * 3, [v * dx for v in lo]))
    t_setup = time.perf_counter()
    from ibamr_amd.slab import Slab
    X = make_markers(cfg["markers"], cfg["M"], Slab([N, N, N], 1, 0, g), 1234, dev)
    X = torch.remainder(X, 1.0).contiguous()
    if args.marker_order == "cell":
        # the level's local numbering (LDataManager::computeNodeDistribution,
        # LDataManager.cpp:2874-2892): patch by patch, cell by cell in box order
        c = torch.clamp((X * N).floor().long(), 0, N - 1)
        t, r = c // n, c % n
        pid = (t[:, 2] * P + t[:, 1]) * P + t[:, 0]
        X = X[torch.argsort((pid * n + r[:, 2]) * n * n + r[:, 1] * n + r[:, 0], stable=True)].contiguous()
        del c, t, r, pid
    M = X.shape[0]
    gen = torch.Generator(device=dev).manual_seed(4321)
    F = torch.rand((M, 3), dtype=torch.float64, device=dev, generator=gen).mul_(2).sub_(1)
    U = torch.zeros((M, 3), dtype=torch.float64, device=dev)
    # the per-patch lists (LIndexSetData::cacheLocalIndices) built on the device in one call
    # (marker order within a patch: the same entries as the reference's cell order, one radix
    # pass by patch instead of four by (patch, cell))
    (ii, _, oi), (si, sx, os_) = le.level_index_lists(ctx, geoms, [0, 0, 0], [N - 1] * 3, X, g, order="markers")
    # one binning serves both sweeps: the ghost-box lists (spread), told which of their
    # entries the interior lists (interp) name (ibtk_le_level_select_interior)
    lvl_s = le.Level.from_flat(ctx, geoms, kernel, X, si, sx, os_)
    lists = {"ii": ii, "oi": oi}
    # each component's patch arrays carved from one allocation (le.alloc_level): the layout the
    # fused level fill + interp reads across patches (ibtk_le_level_fill_interp)
    u = le.alloc_level(geoms, "side", device=dev)
    for per in u:
        for a in per:
            a.uniform_(-1.0, 1.0, generator=gen)
    f = le.alloc_level(geoms, "side", device=dev)
    # algorithmic bytes: the distinct points each patch's ghost-box stencils touch
    S_touched = [0, 0, 0]
    for q, geom in enumerate(geoms):
        if os_[q + 1] == os_[q]:
            continue
        idx_q = si[os_[q]:os_[q + 1]].contiguous()
        xs_q = sx[os_[q]:os_[q + 1]].contiguous()
        mq = le.Markers(ctx).bin(geom, kernel, X, idx_q, xs_q)
        for a, m in enumerate(le.mark_stencils(ctx, mq, kernel, "side", geom, X)):
            S_touched[a] += int(m.sum(dtype=torch.int64).item())
    torch.cuda.synchronize()
    log(f"setup {time.perf_counter() - t_setup:.1f}s: level {P}^3 patches of {n}^3, markers {M}, "
        f"interior entries {oi[-1]}, ghost-box entries {os_[-1]}")
    E = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    acc = {"fill": [], "bin": [], "interp": [], "zero": [], "spread": []}

    dt_move = 0.05 * dx  # |U| <= ~1: markers move <= 1/20 cell per step

    def zero_spread(f):
        if args.unfused_zero:  # the two launches the fused one replaces (A/B)
            lvl_s.zero("side", f)
            lvl_s.spread("side", f, F, X)
        else:
            lvl_s.zero_spread("side", f, F, X)

    # the level's ghost fill fused into the interp (ibtk_le_level_fill_interp: each ghost point
    # read in the neighbour patch the fill copies it from); --unfused-fill: the two calls
    def fill():
        if args.unfused_fill:
            lvl_s.fill_ghosts("side", u)

    def interp():
        if args.unfused_fill:
            lvl_s.interp("side", u, U, X)
        else:
            lvl_s.fill_interp("side", u, U, X)

    def step(record):
        if args.move:
            return step_move(record)
        if record:
            E[0].record()
        fill()
        if record:
            E[1].record()
        if args.full_bin:
            lvl_s.bin(X)
            binning["full"] += 1
        else:
            lvl_s.rebin(X)  # the same lists (between regrids): from the previous order
            binning["rebin"] += 1
        lvl_s.select_interior(M, lists["ii"], lists["oi"])
        if record:
            E[2].record()
        interp()
        if record:
            E[3].record()
            E[4].record()  # zero f: fused into the spread (ibtk_le_level_zero_spread)
        zero_spread(f)
        if record:
            E[5].record()

    nstep = {"k": 0}
    binning = {"full": 0, "rebin": 0}
    # Between regrids the per-patch lists are kept (LIndexSetData between regrids): a marker
    # may drift at most the ghost width's spare cells (g - W/2, LDataManager.cpp:167
    # CFL_WIDTH) from the cell it was listed in, or a patch would miss its spread or
    # interpolate outside its ghost box.  Bounded up front: |U| <= max|u| = 1 (u uniform in
    # [-1, 1]; the closed-form kernels' weights are >= 0 and sum to 1), so a step moves a
    # marker at most dt / dx = 0.05 cells a dim, and the lists serve K - 1 updates; a cadence
    # beyond the slack is refused.  Checked on the device as well, at each regrid, on the
    # positions just before they are wrapped and re-listed (no host sync in the step),
    # reported as config.drift_within_slack.
    slack = g - KERNEL_HALF_WIDTH.get(kernel, 2)
    if args.move and args.regrid_every > 1 and (args.regrid_every - 1) * 0.05 > slack:
        raise SystemExit(f"--regrid-every {args.regrid_every}: {args.regrid_every - 1} updates of up to 0.05 "
                         f"cells exceed the lists' drift slack of {slack} cell(s)")
    # (scratch allocated once: at a regrid in the timed steps fresh 240-MB temporaries cost a
    # 30-140 ms allocation stall, profiles/r06/cfg5_move_trace.txt)
    lazy = args.move and args.regrid_every > 1
    cell_at_regrid = torch.floor(X * N) if lazy else None
    drift_tmp = torch.empty_like(X) if lazy else None
    drift_bad = torch.empty(X.shape, dtype=torch.bool, device=dev) if lazy else None
    drift_flag = torch.zeros(1, dtype=torch.bool, device=dev)

    def cells_of(out):
        torch.mul(X, N, out=out)
        out.floor_()

    def check_drift():
        cells_of(drift_tmp)
        drift_tmp.sub_(cell_at_regrid).abs_()
        torch.gt(drift_tmp, slack, out=drift_bad)
        drift_flag.logical_or_(drift_bad.any())

    if lazy:
        # once outside the timed steps: the first launch of each torch kernel loads its code
        # object (a 113-ms hipLaunchKernel at the first regrid in the timed steps otherwise,
        # profiles/r06/cfg5_r10_stall.txt); the warm-up's regrid skips the check
        check_drift()

    def step_move(record):
        # a moving step on the level: interp at the current positions (the interior lists
        # binned there), X += dt U, spread at the new positions.  At a regrid step (every
        # --regrid-every k-th; IBHierarchyIntegrator's regrid_interval) the positions are
        # wrapped and the per-patch lists rebuilt (LIndexSetData's lists after the
        # redistribution; ibtk_le_level_index_lists, one device pass) and binned afresh; between regrids
        # the lists stay (the markers drift within the ghost width's slack,
        # LDataManager.cpp:167) and are re-binned at the new positions (ibtk_le_markers_rebin)
        at_regrid = nstep["k"] % args.regrid_every == 0
        nstep["k"] += 1
        if record:
            E[0].record()
        fill()
        if record:
            E[1].record()
        interp()
        if record:
            E[2].record()
        le.position_update(ctx, "euler", dt_move, X, U, out=X)
        if at_regrid and args.regrid_every > 1 and nstep["k"] > 1:
            check_drift()  # the drift since the last regrid, before the wrap
        if at_regrid:
            # beginDataRedistribution's wrap into the periodic domain (LDataManager.cpp:1385-1399)
            le.wrap_positions(ctx, X, [0.0, 0.0, 0.0], [1.0, 1.0, 1.0])
            (ii2, _, oi2), (si2, sx2, os2) = le.level_index_lists(ctx, geoms, [0, 0, 0], [N - 1] * 3, X, g,
                                                                  order="markers")
            lists.update(ii=ii2, oi=oi2)
            if lazy:  # the drift check's reference cells
                cells_of(cell_at_regrid)
            lvl_s.relist(si2, sx2, os2).bin(X)
            binning["full"] += 1
        else:
            lvl_s.rebin(X)
            binning["rebin"] += 1
        lvl_s.select_interior(M, lists["ii"], lists["oi"])
        if record:
            E[3].record()
            E[4].record()
        zero_spread(f)
        if record:
            E[5].record()

    for _ in range(args.warmup):
        step(False)
    ctx.synchronize()
    torch.cuda.synchronize()
    binning.update(full=0, rebin=0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed_binning = dict(binning)
    for _ in range(max(3, min(args.steps, 10))):
        step(True)
        torch.cuda.synchronize()
        acc["fill"].append(E[0].elapsed_time(E[1]))
        if args.move:  # E1-E2 interp, E2-E3 update + lists + bin
            acc["interp"].append(E[1].elapsed_time(E[2]))
            acc["bin"].append(E[2].elapsed_time(E[3]))
        else:
            acc["bin"].append(E[1].elapsed_time(E[2]))
            acc["interp"].append(E[2].elapsed_time(E[3]))
        acc["zero"].append(E[3].elapsed_time(E[4]))
        acc["spread"].append(E[4].elapsed_time(E[5]))
    ctx.enable_timing(True)
    kt = {"interp": [], "spread": []}
    for _ in range(3):
        interp()
        ctx.synchronize()
        kt["interp"].append(ctx.last_kernel_ms())
        zero_spread(f)
        ctx.synchronize()
        kt["spread"].append(ctx.last_kernel_ms())
    ctx.enable_timing(False)
    mean = lambda v: sum(v) / len(v)
    k_i, k_s = mean(kt["interp"]), mean(kt["spread"])
    lds = lds_atomic(ctx, lambda: zero_spread(f), k_s)
    # per entry X and Q/F (24 + 24 B), per touched point 8 B (interp) or 16 B (spread);
    # the touched points are those of the ghost-box lists (an upper bound for interp's)
    B_i = M * 48 + 8 * sum(S_touched)
    # the spread into the zeroed f (one sweep) writes every point of f and reads none
    B_s = os_[-1] * 48 + 8 * sum(a.numel() for per in f for a in per)
    dominant = "spread" if k_s >= k_i else "interp"
    achieved = (B_s / (k_s * 1e-3) if dominant == "spread" else B_i / (k_i * 1e-3)) / 1e9
    return {
        "metric": METRIC, "value": 2.0 * M * args.steps / elapsed, "unit": "marker-ops/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": cfg["desc"], "kernel": kernel, "grid": [N, N, N], "markers": M,
                   "parallelism": "one GPU", "patches": [P, P, P], "patch_cells": [n, n, n], "ghost": g,
                   "marker_order": args.marker_order, "move": args.move,
                   "regrid_every": args.regrid_every if args.move else None,
                   "drift_within_slack": ((not bool(drift_flag.item())) if args.move and args.regrid_every > 1
                                          else None),
                   "bin": binning_label(timed_binning, "ibtk_le_level_bin"),
                   "step": ("level ghost fill and interp(3 comps) in one launch + position update + "
                            + (f"at every {args.regrid_every}-th step (regrid) " if args.regrid_every > 1 else "")
                            + "positions wrapped and per-patch lists rebuilt (ibtk_le_level_index_lists, on the device) and binned"
                            + ("; between regrids the lists kept and re-binned at the new positions"
                               if args.regrid_every > 1 else "")
                            + " + interior entries selected + zero f and spread(3 comps) in one launch" if args.move else
                            "bin(ghost-box lists; the interior lists select interp's entries) + "
                            + ("level ghost fill + interp(3 comps)" if args.unfused_fill else
                               "level ghost fill and interp(3 comps) in one launch (ibtk_le_level_fill_interp: ghost points "
                               "read in the neighbour patches)") +
                            " + zero f and spread(3 comps) in one launch (ibtk_le_level_zero_spread); stationary markers, "
                            "per-patch lists built once at setup (LIndexSetData between regrids), one launch per sweep over "
                            "the 512 patches")},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes": {"interp": B_i, "spread": B_s}, "kernel_ms": {"interp": k_i, "spread": k_s},
                     "kernel_note": KERNEL_NOTE, "lds_atomic": lds},
        "cpu_baseline": None,
        "breakdown_ms": {k: mean(v) for k, v in acc.items()},
        "touched_points": S_touched,
    }


def rehearsal():
    """IBTK_BENCH_BACKEND=gloo with IBTK_BENCH_DEVICE set: every rank on that one GPU, the
    exchanges over gloo staged through the host (a wiring check, not the metric)."""
    return os.environ.get("IBTK_BENCH_BACKEND") == "gloo" and "IBTK_BENCH_DEVICE" in os.environ


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, visible=None, poll_s=0.2):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): one child process per rank,
    as torch.distributed.run would start them -- RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous
    at 127.0.0.1 -- each on its own GPU (cuda:LOCAL_RANK), rank 0 printing the line.  Refuses
    (exit status 2, before any GPU call) when fewer than N GPUs are visible, unless the one-GPU
    gloo rehearsal is asked for (rehearsal()); never falls back to fewer ranks.  If a rank fails,
    the others are stopped and its exit status is returned."""
    import subprocess
    if visible is None:
        import torch
        visible = torch.cuda.device_count()  # counts devices without initialising the GPU
    if visible < n and not rehearsal():
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {visible} (for a one-GPU rehearsal set "
              f"IBTK_BENCH_BACKEND=gloo IBTK_BENCH_DEVICE=0)", file=sys.stderr, flush=True)
        return 2
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        # rank 0's stdout is the line; the other ranks' goes to stderr
        procs.append(subprocess.Popen([sys.executable] + argv, env=env, stdout=None if r == 0 else 2))
    code = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and code == 0:
                code = rc if rc > 0 else 1
                for q in live:  # a failed rank: the others would wait for it forever
                    q.kill()
        if live:
            time.sleep(poll_s)
    return code


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg4", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--unfused-zero", action="store_true",
                    help="zero f's ghosts (cfg5: all of f) and spread as two launches instead of one "
                         "(ibtk_le_zero_ghosts_spread / ibtk_le_level_zero_spread; A/B)")
    ap.add_argument("--unfused-fill", action="store_true",
                    help="fill u's periodic ghosts with their own passes, then interp (instead of "
                         "ibtk_le_fill_interp reading the ghost points at their periodic images; A/B)")
    ap.add_argument("--spread-into", default="zero", choices=["zero", "existing"],
                    help="zero: f set to 0 (ghosts included) and spread into, as LDataManager::spread hands "
                         "f to LEInteractor::spread (LDataManager.cpp:596; ibtk_le_zero_spread, one sweep); "
                         "existing: f += S F into the current values, ghosts zeroed (ibtk_le_zero_ghosts_spread)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-rebin", action="store_true", help="bin once outside the timed loop")
    ap.add_argument("--full-bin", action="store_true",
                    help="bin every step from scratch (device radix sort of all keys) instead of re-binning "
                         "from the previous order (ibtk_le_markers_rebin)")
    ap.add_argument("--solo-slab", type=int, default=0, metavar="S",
                    help="projection aid (one GPU, not a scaling measurement): run rank 0's slab of an S-way z "
                         "split alone, its z ghosts wrapped locally instead of exchanged")
    ap.add_argument("--spread-mode", default="sum", choices=["sum", "markers"],
                    help="N > 1: z ghost-region sum of the grid (sum) or the reference's ghost markers (markers)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="diagnostic sweep overrides (ibtk_le_ctx_tune: heavy, seg_items, split_target)")
    ap.add_argument("--layout", default="packed", choices=["aligned", "packed"],
                    help="Eulerian arrays: rows padded to 128 B (aligned) or SAMRAI's packed layout")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: exchange the ghost planes before interp / after spread instead of overlapping "
                         "them with the interior sweep items")
    ap.add_argument("--marker-order", default="cell", choices=["cell", "random"],
                    help="storage order of the markers: 'cell' = sorted by cell (z, y, x), the order "
                         "LDataManager's local numbering gives after redistribution (SURVEY.md 8d); "
                         "'random' = generation order")
    ap.add_argument("--single-patch", action="store_true",
                    help="cfg5 on one 512^3 patch instead of the 8^3-patch level")
    ap.add_argument("--move", action="store_true",
                    help="a full explicit coupling step: interp, X += dt U (ibtk_le_position_update), "
                         "migrate the slab leavers (N > 1), re-bin, spread")
    ap.add_argument("--regrid-every", type=int, default=1, metavar="K",
                    help="with --move: migrate (and with --renumber redistribute) every K-th step only, the "
                         "reference's lazy cadence (regrid_interval); between regrids the markers keep their rank "
                         "and rows, drift at most the ghost width's spare cell past their slab (checked on the "
                         "device) and the binning is a re-binning")
    ap.add_argument("--renumber", action="store_true",
                    help="with --move: after the migration, redistribute every step -- the level's local "
                         "numbering, node offsets, nonlocal nodes and the LData reorder (slab.redistribute; "
                         "the reference does this at regrid, LDataManager.cpp:1504-1959)")
    args = ap.parse_args()
    if args.renumber and not args.move:
        raise SystemExit("--renumber needs --move")
    if args.renumber and CONFIGS[args.config].get("patches") and not args.single_patch:
        raise SystemExit("--renumber: slab configurations only (cfg5's level: --single-patch)")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks here, before anything touches the GPU
        raise SystemExit(launch_ranks(args.gpus, [str(Path(__file__).resolve())] + sys.argv[1:]))

    import torch
    cfg = CONFIGS[args.config]
    kernel = args.kernel or cfg["kernel"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
    # IBTK_BENCH_DEVICE / IBTK_BENCH_BACKEND=gloo: a multi-rank rehearsal with every
    # rank on one GPU (exchanges staged through the host); the default is one rank
    # per GPU over RCCL
    local_dev = int(os.environ.get("IBTK_BENCH_DEVICE", local))
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if os.environ.get("IBTK_BENCH_BACKEND", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    if cfg.get("patches") and not args.single_patch and world == 1:
        out = run_level(args, cfg, kernel, dev)
        if not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, kernel, args.cpu_seconds)
            except Exception as e:  # the baseline must never hide the GPU result
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
        return

    from ibamr_amd import le
    from ibamr_amd.slab import (GhostMarkers, Slab, SlabExchange, migrate, redistribute, update_and_migrate,
                                update_and_migrate_fixed)

    N = cfg["N"]
    ghost = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    # ghost planes exchanged per face: the stencils' reach W/2 (= ghost - 1) while every
    # marker sits in its slab (stationary, or migrated every step); the full ghost width
    # when they drift up to a cell past it between regrids (--regrid-every k > 1)
    width = ghost if (args.move and args.regrid_every > 1) else max(1, ghost - 1)
    slab = Slab([N, N, N], world, rank, ghost, align=16 if args.layout == "aligned" else 0, width=width)
    xslab = slab  # the slab the exchanges see
    if args.solo_slab > 1:
        if world > 1:
            raise SystemExit("--solo-slab runs on one rank")
        S = args.solo_slab
        slab = Slab([N, N, N], S, 0, ghost, align=16 if args.layout == "aligned" else 0)
        # the same planes, periodic in z on their own: the local fill / fold stand in for
        # the exchange (same arrays, same passes); the RCCL transfers are not modelled
        xslab = Slab([N, N, N // S], 1, 0, ghost, L=(1.0, 1.0, 1.0 / S),
                     align=16 if args.layout == "aligned" else 0)
    geom = slab.geometry()
    ctx = le.Context(local_dev)
    for kv in args.tune:
        ctx.tune(kv.split("=")[0], int(kv.split("=")[1]))

    t_setup = time.perf_counter()
    X = make_markers(cfg["markers"], cfg["M"], slab, 1234, dev)
    if args.marker_order == "cell":
        # local numbering in cell order (LDataManager::computeNodeDistribution,
        # LDataManager.cpp:2839-3027: interior markers in patch-cell iteration order)
        ci = [torch.clamp((X[:, d] / slab.dx[d]).floor().long(), 0, N - 1) for d in range(3)]
        X = X[torch.argsort((ci[2] * N + ci[1]) * N + ci[0])].contiguous()
        del ci
    M_local = X.shape[0]
    gen = torch.Generator(device=dev).manual_seed(4321 + rank)
    F = torch.rand((M_local, 3), dtype=torch.float64, device=dev, generator=gen).mul_(2).sub_(1)
    U = torch.zeros((M_local, 3), dtype=torch.float64, device=dev)
    # N > 1 moving steps: fixed-capacity marker arrays whose length stays on the device
    # (slab.update_and_migrate_fixed; no host sync in the step)
    fixed = world > 1 and args.move and not args.renumber and args.spread_mode == "sum"
    n_dev, send_cap = None, 0
    if fixed:
        cap = M_local + max(M_local // 8, 65536)
        send_cap = max(M_local // 32, 16384)
        pad = lambda t: torch.cat([t, torch.zeros((cap - M_local, 3), dtype=t.dtype, device=dev)]).contiguous()
        X, F, U = pad(X), pad(F), pad(U)
        n_dev = torch.tensor([M_local], dtype=torch.int32, device=dev)
    # Lagrangian indices (globally unique: rank-major generation order) for --renumber
    lag = (torch.arange(M_local, dtype=torch.int32, device=dev) * world + rank) if args.renumber else None
    u = geom.alloc("side", device=dev)
    for a in u:
        a.uniform_(-1.0, 1.0, generator=gen)
    f = geom.alloc("side", device=dev)
    ex_u = SlabExchange(xslab, u, ctx)
    ex_f = SlabExchange(xslab, f, ctx)
    if not args.no_overlap:
        ex_u.cut_items()  # sweep items cut at the slab faces (N > 1)
    bins = le.Markers(ctx)
    gm = GhostMarkers(slab) if args.spread_mode == "markers" and world > 1 else None
    # the binned list: own markers, or (ghost-marker mode) own + the neighbours'
    # markers near the slab faces, exchanged with their forces every step
    cur = {"X": X, "F": F, "U": U}

    binned = {"rows": None, "changed": False}
    # the lazy cadence's bound: between regrids a marker may drift at most `slack` cells
    # past its slab (the ghost width's spare plane, LDataManager.cpp:167 CFL_WIDTH), checked
    # on the device after every update and reported after the run (no host sync per step)
    slack = ghost - max(1, ghost - 1)
    drift_flag = torch.zeros(1, dtype=torch.bool, device=dev)

    def check_drift(Xc, n_rows=None):
        cz = torch.floor(Xc[:, 2] / slab.dx[2])
        bad = (cz < slab.z0 - slack) | (cz >= slab.z1 + slack)
        for d in range(2):
            c = torch.floor(Xc[:, d] / slab.dx[d])
            bad |= (c < -slack) | (c >= N + slack)
        if n_rows is not None:  # a fixed-capacity array: the rows in use (device count)
            bad &= torch.arange(Xc.shape[0], device=Xc.device) < n_rows
        drift_flag.logical_or_(bad.any())

    binning = {"full": 0, "rebin": 0}  # what the binning did (the record's "bin" label)

    def bin_step():
        if fixed:
            bins.bin_count(geom, kernel, X, n_dev)
            binning["full"] += 1
            cur.update(X=X, F=F, U=U)
            return
        if gm is None:
            # the same rows as at the last binning (no migration changed the list): re-bin
            # from the previous order (ibtk_le_markers_rebin, exact); else bin afresh
            if not args.full_bin and binned["rows"] == X.shape[0] and not binned["changed"]:
                bins.rebin(X)
                binning["rebin"] += 1
            else:
                bins.bin(geom, kernel, X)
                binning["full"] += 1
                binned["rows"] = X.shape[0]
                binned["changed"] = False
            cur.update(X=X, F=F, U=U)
            return
        Xa, Fa, _ = gm.exchange(X, F)
        bins.bin(geom, kernel, Xa)
        binning["full"] += 1
        Ua = cur["U"] if cur["U"].shape == Xa.shape else torch.empty_like(Xa)
        cur.update(X=Xa, F=Fa, U=Ua)

    bin_step()
    # exact algorithmic bytes: distinct side points touched by the clipped stencils
    masks = le.mark_stencils(ctx, bins, kernel, "side", geom, cur["X"])
    S_touched = [int(m.sum(dtype=torch.int64).item()) for m in masks]
    del masks
    torch.cuda.synchronize()
    M_total = M_local
    if world > 1:
        t = torch.tensor([M_local], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        M_total = int(t.item())
    log(f"setup {time.perf_counter() - t_setup:.1f}s: rank {rank} markers {M_local} of {M_total}, "
        f"slab z[{slab.z0},{slab.z1}), touched {S_touched}")

    E = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    acc = {"bin": [], "interp": [], "zero": [], "spread": []}

    dt_move = 0.05 * slab.dx[0]  # |U| <= ~1: markers move <= 1/20 cell per step

    # the periodic ghost fill of u fused into the interp's sweep (ibtk_le_fill_interp: the
    # ghost points read at their periodic images, x/y/z on one rank, x/y on a slab whose z
    # ghost planes come from its neighbours); --unfused-fill: the fill passes, then interp
    fused_fill = not args.unfused_fill

    def interp_call(Ub, Xb):
        if fused_fill:
            le.fill_interp(ctx, bins, kernel, "side", geom, u, Ub, Xb, periodic=[1, 1, 1 if world == 1 else 0])
        else:
            le.interp(ctx, bins, kernel, "side", geom, u, Ub, Xb)

    def interp_with_fill():
        # N > 1: the interior sweep items run while the z ghost planes are in flight
        Xb, Ub = cur["X"], cur["U"]
        if args.no_overlap:
            ex_u.halo_fill(local=not fused_fill)
            interp_call(Ub, Xb)
        else:
            ex_u.halo_fill(lambda: interp_call(Ub, Xb), local=not fused_fill)
        if Ub is not U:
            U.copy_(Ub[:U.shape[0]])  # the own markers' velocities (ghost markers' discarded)

    # f's zeroing fused into the spread's sweep: --spread-into zero (default), the whole
    # of f (ibtk_le_zero_spread: items start every owned point from 0 and read nothing);
    # existing, the ghosts (ibtk_le_zero_ghosts_spread).  --unfused-zero: the zeroing
    # (zero_step) and the spread as separate launches
    def spread_call(Fb, Xb):
        if args.unfused_zero:
            le.spread(ctx, bins, kernel, "side", geom, f, Fb, Xb)
        elif args.spread_into == "zero":
            le.zero_spread(ctx, bins, kernel, "side", geom, f, Fb, Xb)
        else:
            le.zero_ghosts_spread(ctx, bins, kernel, "side", geom, f, Fb, Xb)

    def spread_with_sum():
        Xb, Fb = cur["X"], cur["F"]

        def spread():
            spread_call(Fb, Xb)
        if gm is not None:
            # ghost markers: every rank spreads what reaches its own planes, no z
            # exchange of the grid; x/y periodic ghosts fold locally
            spread()
            ex_f.local_fold([1, 1, 0])
            return
        # N > 1: the boundary items first, then the interior ones while the ghost
        # planes are in flight
        if args.no_overlap:
            spread()
            ex_f.ghost_sum()
        else:
            ex_f.ghost_sum(spread)

    def zero_step():
        if args.unfused_zero:
            if args.spread_into == "zero":
                for a in f:
                    a.zero_()
            else:
                le.zero_ghosts(ctx, geom, "side", f)

    nstep = {"k": 0}

    def step_move(record):
        # interp -> X += dt U -> migrate -> bin -> spread: one bin per step, as in
        # IBMethod's explicit loop (interpolateVelocity, eulerStep, spreadForce).  The
        # markers migrate (and are renumbered) at regrid steps only: every step by
        # default, every k-th with --regrid-every k (IBHierarchyIntegrator's
        # regrid_interval, IBHierarchyIntegrator.cpp:495-508); between regrids they keep
        # their rank and rows, and the binning is a re-binning of the same list
        nonlocal X, F, U, lag, n_dev
        at_regrid = nstep["k"] % args.regrid_every == 0
        nstep["k"] += 1
        if record:
            E[0].record()
        interp_with_fill()
        if record:
            E[1].record()
        if not at_regrid:
            le.position_update(ctx, "euler", dt_move, X, U, out=X)
            if world > 1:  # the slab-ownership slack (one rank: the periodic box is the slab)
                check_drift(X, n_dev if fixed else None)
        elif fixed:
            X, (F,), n_dev = update_and_migrate_fixed(slab, ctx, "euler", dt_move, X, U, [F], n_dev, send_cap)
            binned["changed"] = True
        elif world > 1:
            # fused on the device: update, wrap, owner classes, stable partition;
            # the leavers to the z-neighbours (slab.update_and_migrate)
            if lag is None:
                X, (F,) = update_and_migrate(slab, ctx, "euler", dt_move, X, U, [F])
            else:
                X, (F, lagf) = update_and_migrate(slab, ctx, "euler", dt_move, X, U, [F, lag.to(torch.float64)])
                lag = lagf.to(torch.int32)
            if U.shape != X.shape:
                U = torch.empty_like(X)
            binned["changed"] = True
        else:
            le.position_update(ctx, "euler", dt_move, X, U, out=X)
        if lag is not None and at_regrid:
            # the level's numbering and the LData reorder (cell order again after the move)
            d = redistribute(slab, ctx, X, [F], lag)
            X, F, lag = d.X, d.fields[0], d.lag
            binned["changed"] = True
        bin_step()
        if record:
            E[2].record()
        zero_step()
        if record:
            E[3].record()
        spread_with_sum()
        if record:
            E[4].record()

    def step(record):
        if args.move:
            return step_move(record)
        if record:
            E[0].record()
        if not args.no_rebin or gm is not None:
            bin_step()
        if record:
            E[1].record()
        interp_with_fill()
        if record:
            E[2].record()
        zero_step()
        if record:
            E[3].record()
        spread_with_sum()
        if record:
            E[4].record()

    def collect():
        # interp / spread include their ghost exchange (overlapped when N > 1)
        torch.cuda.synchronize()
        if args.move:  # E0-E1 fill + interp, E1-E2 update + migrate + bin
            acc["interp"].append(E[0].elapsed_time(E[1]))
            acc["bin"].append(E[1].elapsed_time(E[2]))
        else:
            acc["bin"].append(E[0].elapsed_time(E[1]))
            acc["interp"].append(E[1].elapsed_time(E[2]))
        acc["zero"].append(E[2].elapsed_time(E[3]))
        acc["spread"].append(E[3].elapsed_time(E[4]))

    # N > 1 overlap self-check on this backend (RCCL in the product), before the timed
    # steps: the overlapped exchanges (interior sweep items running while the ghost
    # planes are in flight on the communicator's stream) must give the bits of the
    # sequential form on every rank; if they do not, the timed steps use the
    # sequential exchange (and the record says so)
    overlap_check = None
    if world > 1 and not args.no_overlap and gm is None:
        Xb = cur["X"]
        Uo, Us = torch.empty_like(cur["U"]), torch.empty_like(cur["U"])
        ex_u.halo_fill(lambda: interp_call(Uo, Xb), local=not fused_fill)
        ex_u.halo_fill(local=not fused_fill)
        interp_call(Us, Xb)
        fo = []
        for overlapped in (True, False):
            for a in f:
                a.zero_()
            if overlapped:  # the timed steps' form
                ex_f.ghost_sum(lambda: spread_call(cur["F"], Xb))
            else:
                spread_call(cur["F"], Xb)
                ex_f.ghost_sum()
            fo.append([a.clone() for a in f])
        same = torch.equal(Uo, Us) and all(torch.equal(a, b) for a, b in zip(*fo))
        t = torch.tensor([0 if same else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        del fo, Uo, Us
        if int(t.item()) == 0:
            overlap_check = "bitwise equal to the sequential exchange on every rank"
        else:
            overlap_check = "DIFFERS from the sequential exchange: timed with the sequential exchange"
            args.no_overlap = True
            log("overlap self-check FAILED: overlapped exchange differs from the sequential one; "
                "the timed steps use the sequential exchange")

    for _ in range(args.warmup):
        step(False)
    ctx.synchronize()

    # timed region: barrier + sync on both sides, exactly K steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    binning.update(full=0, rebin=0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    torch.cuda.synchronize()
    timed_binning = dict(binning)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ctx.synchronize()

    # per-kernel breakdown on the context stream (separate instrumented steps)
    for _ in range(max(3, min(args.steps, 10))):
        step(True)
        collect()
    # the sweep kernels alone: HIP events the library records around each
    # launch on the context stream (ibtk_le_ctx_last_kernel_ms)
    ctx.enable_timing(True)
    kt = {"interp": [], "spread": []}
    for _ in range(3):
        ex_u.halo_fill(local=not fused_fill)
        interp_call(cur["U"], cur["X"])
        ctx.synchronize()
        kt["interp"].append(ctx.last_kernel_ms())
        zero_step()
        spread_call(cur["F"], cur["X"])
        ctx.synchronize()
        kt["spread"].append(ctx.last_kernel_ms())
    ctx.enable_timing(False)

    ms_per_step = 1e3 * elapsed / args.steps
    value = 2.0 * M_total * args.steps / elapsed
    lds = lds_atomic(ctx, lambda: le.spread(ctx, bins, kernel, "side", geom, f, cur["F"], cur["X"]),
                     sum(kt["spread"]) / len(kt["spread"]))

    def mean(v):
        return sum(v) / len(v)

    t_i, t_s = mean(acc["interp"]), mean(acc["spread"])
    k_i, k_s = mean(kt["interp"]), mean(kt["spread"])
    B_i = M_local * 48 + 8 * sum(S_touched)
    # the spread reads and writes the touched points; into a zeroed f (the default) it
    # writes every point of f once and reads none
    B_s = M_local * 48 + (8 * sum(a.numel() for a in f) if args.spread_into == "zero" else 16 * sum(S_touched))
    dominant = "spread" if k_s >= k_i else "interp"
    achieved = (B_s / (k_s * 1e-3) if dominant == "spread" else B_i / (k_i * 1e-3)) / 1e9
    pair = (B_i + B_s) / ((t_i + t_s) * 1e-3) / 1e9
    # HBM traffic per launch of the dominant kernel from the rocprofv3 PMC passes of
    # tools/pmc_traffic.sh (2 x FETCH_SIZE + WRITE_SIZE: FETCH_SIZE counts half the
    # bytes of 8- and 16-byte-per-lane reads on gfx950, profiles/r02b/
    # fetch_calibration.json), used only if it profiled this very build
    traffic, traffic_note = None, "no PMC profile of this build"
    pmc = ROOT / "profiles" / f"pmc_{args.config}_{kernel}_{world}gpu.json"
    if pmc.exists():
        try:
            from ibamr_amd.build import source_hash
            rec = json.loads(pmc.read_text())
            if rec.get("build") == source_hash():
                traffic = rec.get("per_launch_bytes", {}).get(dominant)
                traffic_note = (f"PMC {pmc.relative_to(ROOT)}: 2 x FETCH_SIZE + WRITE_SIZE per launch, "
                                f"build {rec['build']}")
            else:
                traffic_note = f"PMC {pmc.relative_to(ROOT)} profiled build {rec.get('build')}, not this one"
        except Exception as e:
            traffic_note = f"PMC record unreadable: {e!r}"

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(cfg, kernel, args.cpu_seconds)
        except Exception as e:  # the baseline must never hide the GPU result
            cpu = {"value": None, "error": repr(e)}

    zname = "zero f" if args.spread_into == "zero" else "zero ghosts"
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "marker-ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": cfg["desc"], "kernel": kernel, "grid": [N, N, N], "markers": M_total,
                   "parallelism": f"z-slab x{world}", "ghost": ghost, "marker_order": args.marker_order, "layout": args.layout, "spread_mode": args.spread_mode if world > 1 else "one rank",
                   "solo_slab": args.solo_slab or None,
                   "bin": binning_label(timed_binning, "ibtk_le_markers_bin" + ("_count" if fixed else "")),
                   "move": args.move, "renumber": args.renumber,
                   "spread_into": ("zeroed f (LDataManager::spread, LDataManager.cpp:596)" if args.spread_into == "zero"
                                   else "f += S F, ghosts zeroed"),
                   "regrid_every": args.regrid_every if args.move else None,
                   "exchange_width": slab.width if world > 1 else None,
                   "drift_within_slack": ((not bool(drift_flag.item())) if args.move and args.regrid_every > 1
                                          and world > 1 else None),
                   "migration": ("fixed-capacity, device counts, no host sync" if fixed else
                                 "counts read by the host" if world > 1 and args.move else None), "overlap": world > 1 and not args.no_overlap,
                   "overlap_check": overlap_check,
                   "step": ("ghost fill + interp(3 comps) + position update + " +
                            (f"at every {args.regrid_every}-th step (regrid) " if args.regrid_every > 1 else "") +
                            "migrate + " +
                            ("redistribute (numbering + nonlocal nodes + reorder) + " if args.renumber else "") +
                            "bin + " + zname + " + "
                            "spread(3 comps) + ghost sum" if args.move else
                            "bin + ghost fill + interp(3 comps) + " + zname + " + spread(3 comps) + ghost sum") +
                           ("" if args.unfused_zero else
                            ("; f's zeroing fused into the spread sweep (ibtk_le_zero_spread: f written once, not read)"
                             if args.spread_into == "zero" else
                             "; the ghost zeroing fused into the spread sweep (ibtk_le_zero_ghosts_spread)")) +
                           ("" if args.unfused_fill else
                            "; the periodic ghost fill fused into the interp sweep (ibtk_le_fill_interp)")},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes per launch (PMC)", "traffic_note": traffic_note,
                     "algorithmic_bytes": {"interp": B_i, "spread": B_s},
                     "kernel_ms": {"interp": k_i, "spread": k_s},
                     "kernel_note": KERNEL_NOTE,
                     "pair_achieved": pair, "pair_frac": pair / HBM_PEAK_GBS, "lds_atomic": lds},
        "cpu_baseline": cpu,
        "breakdown_ms": {k: mean(v) for k, v in acc.items()},
        "touched_points": S_touched,
    }
    if args.solo_slab > 1:  # a projection aid, never the metric
        out["projection"] = {"slabs": args.solo_slab, "per_rank_value": value,
                             "value_if_exchanges_hidden": value * args.solo_slab,
                             "note": "rank 0's slab alone on one GPU, z ghosts wrapped locally; RCCL not modelled"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
