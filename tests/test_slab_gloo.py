"""Multi-rank slab decomposition on CPU (gloo, world size 2 and 4).

Checks the z-halo fill and the ghost-region sum of ibamr_amd.slab against the
global periodic answer.  The local x/y periodic pieces, which run as HIP kernels
in the product, are replaced here by a numpy restatement of the same kernel
semantics (ibamr_amd/csrc/le_aux.hip, k_ghost): fill wraps every periodic dim
of a ghost point at once; fold walks dims slowest first, region d = (dims < d
any, dim d ghost, dims > d interior if periodic, any if not), one source per
destination per pass.
Values are small integers so every sum is exact and the comparison is bitwise.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _interior(slab, comp):
    """unique (interior) index ranges per dim in array coordinates, for dims x, y, z."""
    g = slab.ghost
    return [(g, g + slab.N[0]), (g, g + slab.N[1]), (g, g + slab.nz)]


def _np_local(arrays, periodic, slab, mode):
    for c, t in enumerate(arrays):
        a = t.numpy()  # shares memory
        rng = _interior(slab, c)
        shape = a.shape[::-1]  # (nx, ny, nz)
        nd = 3
        if mode == "fill":
            idx = np.indices(shape).reshape(3, -1).T  # (x, y, z)
            for pt in idx:
                inside = all(rng[d][0] <= pt[d] < rng[d][1] for d in range(nd))
                if inside:
                    continue
                # wrap the periodic dims only; a non-periodic ghost coordinate is kept
                src = list(pt)
                moved = False
                for d in range(nd):
                    if periodic[d] and not (rng[d][0] <= pt[d] < rng[d][1]):
                        n = rng[d][1] - rng[d][0]
                        src[d] = rng[d][0] + (pt[d] - rng[d][0]) % n
                        moved = True
                if moved:
                    a[pt[2], pt[1], pt[0]] = a[src[2], src[1], src[0]]
        else:
            for dreg in (2, 1, 0):
                if not periodic[dreg]:
                    continue
                sl = [slice(None)] * 3  # in (x, y, z) order
                for d in range(nd):
                    if d > dreg and periodic[d]:  # non-periodic dims: their ghost layers too
                        sl[d] = slice(*rng[d])
                n = rng[dreg][1] - rng[dreg][0]
                for j in list(range(0, rng[dreg][0])) + list(range(rng[dreg][1], shape[dreg])):
                    dst = rng[dreg][0] + (j - rng[dreg][0]) % n
                    s_src, s_dst = list(sl), list(sl)
                    s_src[dreg], s_dst[dreg] = j, dst
                    a[tuple(s_dst[::-1])] += a[tuple(s_src[::-1])]


def _worker(rank, world, port, N, ghost, out_q, width=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ibamr_amd.slab import Slab, SlabExchange
        slab = Slab([N, N, N], world, rank, ghost, width=width)
        w = slab.width
        # z planes the exchanges cover (array coordinates): the interior and `width`
        # ghost planes per face (the z component's upper block one plane thicker);
        # with one rank every plane (local periodic fill / fold)
        def zcov(c):
            if world == 1:
                return slice(None)
            return slice(ghost - w, ghost + slab.nz + w + (1 if c == 2 else 0))
        geom_shapes = []
        for c in range(3):
            n = [N + 2 * ghost + (1 if d == c else 0) for d in range(2)] + [slab.nz + 2 * ghost + (1 if c == 2 else 0)]
            geom_shapes.append(tuple(reversed(n)))
        rng = np.random.default_rng(100 + rank)
        # ---- halo fill: interior = global field, ghosts garbage
        Gs = [np.random.default_rng(7 + c).integers(-50, 50, (N, N, N)).astype(np.float64) for c in range(3)]
        arrays = []
        for c in range(3):
            a = rng.integers(-1000, 1000, geom_shapes[c]).astype(np.float64)
            zz = np.arange(a.shape[0]) - ghost + slab.z0
            yy = np.arange(a.shape[1]) - ghost
            xx = np.arange(a.shape[2]) - ghost
            full = Gs[c][np.ix_(zz % N, yy % N, xx % N)]
            inner = (slice(ghost, ghost + slab.nz), slice(ghost, ghost + N), slice(ghost, ghost + N))
            a[inner] = full[inner]
            arrays.append(torch.from_numpy(a))
        ex = SlabExchange(slab, arrays, local_fill=lambda arr, per: _np_local(arr, per, slab, "fill"),
                          local_fold=lambda arr, per: _np_local(arr, per, slab, "fold"))
        ex.halo_fill()
        for c in range(3):
            a = arrays[c].numpy()
            zz = np.arange(a.shape[0]) - ghost + slab.z0
            yy = np.arange(a.shape[1]) - ghost
            xx = np.arange(a.shape[2]) - ghost
            expect = Gs[c][np.ix_(zz % N, yy % N, xx % N)]
            assert np.array_equal(a[zcov(c)], expect[zcov(c)]), f"halo_fill rank {rank} comp {c}"
        # ---- ghost sum: every point the exchange covers (interior and ghost) carries a
        # value (the planes beyond `width` hold none, as a stencil never reaches them);
        # the result's interior must equal the sum of all values wrapping onto it
        arrays = []
        for c in range(3):
            a = np.zeros(geom_shapes[c])
            a[zcov(c)] = rng.integers(-20, 20, geom_shapes[c]).astype(np.float64)[zcov(c)]
            arrays.append(torch.from_numpy(a))
        before = [a.numpy().copy() for a in arrays]
        ex = SlabExchange(slab, arrays, local_fill=lambda arr, per: _np_local(arr, per, slab, "fill"),
                          local_fold=lambda arr, per: _np_local(arr, per, slab, "fold"))
        ex.ghost_sum()
        # gather every rank's 'before' arrays to compute the global wrap-sum
        objs = [None] * world
        dist.all_gather_object(objs, (slab.z0, before))
        for c in range(3):
            tot = np.zeros((N, N, N))
            for z0, bl in objs:
                b = bl[c]
                zz = (np.arange(b.shape[0]) - ghost + z0) % N
                yy = (np.arange(b.shape[1]) - ghost) % N
                xx = (np.arange(b.shape[2]) - ghost) % N
                np.add.at(tot, np.ix_(zz, yy, xx), b)
            a = arrays[c].numpy()
            inner = a[ghost:ghost + slab.nz, ghost:ghost + N, ghost:ghost + N]
            assert np.array_equal(inner, tot[slab.z0:slab.z1]), f"ghost_sum rank {rank} comp {c}"
        out_q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        out_q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,width", [(1, None), (2, None), (4, None), (2, 2), (4, 2)])
def test_slab_exchange_gloo(world, width):
    """width None: the ghost width (3) per face; 2: the planes an IB_4 stencil of a marker
    inside the slab reaches (Slab.width)."""
    N, ghost = 16, 3
    if world > 1 and N // world < 2 * ghost + 2:
        N = world * (2 * ghost + 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, ghost, q, width)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    for _ in range(world):
        try:
            results.append(q.get(timeout=120))
        except Exception:
            results.append((-1, "worker died: " + str([p.exitcode for p in procs])))
            break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    bad = [r for r in results if r[1] != "ok"]
    assert not bad, bad[0][1]


def _migrate_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ibamr_amd.slab import Slab, migrate
    slab = Slab([16, 16, 32], world, rank, 3)
    g = torch.Generator().manual_seed(100 + rank)
    M = 500 + 37 * rank
    X = torch.rand((M, 3), dtype=torch.float64, generator=g) * 1.4 - 0.2  # some outside [0, 1): periodic images
    ids = (torch.arange(M, dtype=torch.int64) + 100000 * rank)
    F = torch.rand((M, 3), dtype=torch.float64, generator=g)
    Xn, (idn, Fn) = migrate(slab, X, [ids, F])
    Xn2, (idn2, Fn2) = migrate(slab, X, [ids, F])  # determinism
    ok = torch.equal(Xn, Xn2) and torch.equal(idn, idn2) and torch.equal(Fn, Fn2)
    zc = (Xn[:, 2] / slab.dx[2]).floor().long()
    owned = bool(((zc >= slab.z0) & (zc < slab.z1)).all())
    inbox = bool(((Xn >= 0) & (Xn < 1)).all())
    # leavers-only form: stayers keep their order, arrivals follow
    Xl, (idl, Fl) = migrate(slab, X, [ids, F], cell_order=False)
    zl = (Xl[:, 2] / slab.dx[2]).floor().long()
    owned = owned and bool(((zl >= slab.z0) & (zl < slab.z1)).all())
    zc0 = (torch.remainder(X[:, 2], 1.0) / slab.dx[2]).floor().long()
    stay_ids = ids[(zc0 >= slab.z0) & (zc0 < slab.z1)].tolist()
    ok = ok and idl[:len(stay_ids)].tolist() == stay_ids and sorted(idl.tolist()) == sorted(idn.tolist())
    ok = ok and all(torch.equal(Fl[idl == i], Fn[idn == i]) for i in idl[::50].tolist())
    out_q.put((rank, ok, owned, inbox, idn.tolist(), Xn.numpy().copy(), Fn.numpy().copy(),
               X.numpy().copy(), ids.numpy().copy(), F.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_marker_migration_gloo(world):
    """Every marker ends on the rank owning its (wrapped) cell, exactly once, with
    its fields; local order is cell order; repeated calls give identical results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_migrate_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    all_ids, before = [], {}
    for rank, ok, owned, inbox, idn, Xn, Fn, X, ids, F in res:
        assert ok and owned and inbox, (rank, ok, owned, inbox)
        all_ids += idn
        for i, x, f in zip(ids, X, F):
            before[int(i)] = (np.mod(x, 1.0), f)
        # cell order within the rank
        c = np.floor(Xn / (1.0 / np.array([16, 16, 32]))).astype(np.int64)
        key = (c[:, 2] * 16 + c[:, 1]) * 16 + c[:, 0]
        assert np.all(np.diff(key) >= 0)
    assert sorted(all_ids) == sorted(before)
    for rank, ok, owned, inbox, idn, Xn, Fn, X, ids, F in res:
        for i, x, f in zip(idn, Xn, Fn):
            xb, fb = before[int(i)]
            assert np.allclose(x, xb, atol=1e-15, rtol=0) and np.array_equal(f, fb)


def _ghost_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ibamr_amd.slab import GhostMarkers, Slab
        N, g = [16, 16, 32], 3
        slab = Slab(N, world, rank, g)
        rng = np.random.default_rng(7)
        Xg = rng.uniform(0, 1, (3000, 3))
        Fg = rng.standard_normal((3000, 3))
        ids = np.arange(3000)
        z = Xg[:, 2]
        mine = (z >= slab.z0 * slab.dx[2]) & (z < slab.z1 * slab.dx[2])
        X = torch.from_numpy(Xg[mine])
        F = torch.from_numpy(np.column_stack([Fg[mine], ids[mine]]))  # the id rides along as a field
        out = []
        for rep in range(2):
            Xa, Fa, n_own = GhostMarkers(slab).exchange(X, F)
            out.append((Xa.numpy().copy(), Fa.numpy().copy(), n_own))
        same = np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
        q.put((rank, "ok", slab.z0, slab.z1, out[0], same))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), 0, 0, None, False))


@pytest.mark.parametrize("world", [2, 4])
def test_ghost_marker_exchange_gloo(world):
    """Reference-mode spread exchange (GhostMarkers): each rank ends with its own
    markers first, then exactly the other ranks' markers whose cell lies within
    `ghost` planes beyond its faces (periodic in z, shifted by -+L_z across the
    wrap), with their forces; deterministic on a repeat."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ghost_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    bad = [r for r in res if r[1] != "ok"]
    assert not bad, bad[0][1]
    rng = np.random.default_rng(7)
    Xg = rng.uniform(0, 1, (3000, 3))
    Fg = rng.standard_normal((3000, 3))
    Nz, g = 32, 3
    dz = 1.0 / Nz
    cz = np.clip(np.floor(Xg[:, 2] / dz).astype(int), 0, Nz - 1)
    for rank, _, z0, z1, (Xa, Fa, n_own), same in res:
        assert same
        ids = Fa[:, 3].astype(int)
        own = set(np.nonzero((cz >= z0) & (cz < z1))[0].tolist())
        assert set(ids[:n_own].tolist()) == own and n_own == len(own)
        # ghosts: cells in [z0 - g, z0) and [z1, z1 + g), wrapped
        want = set()
        for i in range(3000):
            if i in own:
                continue
            for shift in (-Nz, 0, Nz):
                c = cz[i] + shift
                if z0 - g <= c < z0 or z1 <= c < z1 + g:
                    want.add((i, shift))
        got = set()
        for k in range(n_own, len(ids)):
            i = ids[k]
            shift = int(round((Xa[k, 2] - Xg[i, 2]) / 1.0)) * Nz
            assert np.array_equal(Xa[k, :2], Xg[i, :2]) and np.array_equal(Fa[k, :3], Fg[i])
            assert abs(Xa[k, 2] - (Xg[i, 2] + shift / Nz)) < 1e-15
            got.add((i, shift))
        assert got == want, (rank, len(got), len(want))
        assert len(ids) - n_own == len(want)


# ---------------------------------------------------------------------------- redistribution
def _redist_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle as ora
        from ibamr_amd.slab import Slab, migrate, redistribute
        N = [12, 10, 32]
        slab = Slab(N, world, rank, 2)
        g = torch.Generator().manual_seed(300 + rank)
        M = 400 + 23 * rank
        X = torch.rand((M, 3), dtype=torch.float64, generator=g)
        X[: M // 4, 2] = (torch.rand(M // 4, dtype=torch.float64, generator=g) * 0.1 - 0.05) % 1.0  # near z = 0
        # just above z = 0: z + L_z - L_z rounds these to 0, the owner's bits must survive
        X[M // 4: M // 4 + 20, 2] = torch.rand(20, dtype=torch.float64, generator=g) * 1e-12
        lag = (torch.randperm(M, generator=g) * world + rank).to(torch.int32)
        F = torch.rand((M, 3), dtype=torch.float64, generator=g)
        Xm, (Fm, lm) = migrate(slab, X, [F, lag.to(torch.float64)], cell_order=False)
        lm = lm.to(torch.int32)
        boxes = [([0, 0, slab.z0], [N[0] - 1, N[1] - 1, slab.z1 - 1])]
        dx = [1.0 / n for n in N]

        def numbering(Xa, la, ghost):  # the oracle stands in for the HIP numbering on CPU
            o, nl, nn = ora.level_node_distribution(Xa.numpy(), la.numpy(), boxes, [0, 0, 0],
                                                    [n - 1 for n in N], [0.0] * 3, dx, ghost)
            return torch.from_numpy(o), nl, nn

        def reorder(order, *arrays):
            return [a[order.long()] for a in arrays]

        def wrap(Xw):  # beginDataRedistribution's wrap (LDataManager.cpp:1385-1399), one period
            L = torch.ones(3, dtype=Xw.dtype)
            Xw = torch.where(Xw < 0, Xw + L, Xw)
            Xw = torch.where(Xw >= L, Xw - L, Xw)
            return torch.minimum(torch.clamp(Xw, min=0.0), L - torch.finfo(Xw.dtype).eps)

        d = redistribute(slab, None, Xm, [Fm], lm, numbering=numbering, reorder=reorder, wrap=wrap)
        ok = torch.equal(d.X, Xm[d.order.long()]) and torch.equal(d.fields[0], Fm[d.order.long()])
        ok = ok and torch.equal(d.lag, lm[d.order.long()])
        q.put((rank, "ok", ok, dict(lag=d.lag.numpy(), offset=d.offset, num_nodes=d.num_nodes,
                                    ghost_lag=d.ghost_lag.numpy(), ghost_petsc=d.ghost_petsc.numpy(),
                                    X=d.X.numpy(), ghost_X=d.ghost_X.numpy()),
               Xm.numpy(), lm.numpy()))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc(), False, None, None, None))


@pytest.mark.parametrize("world", [2, 4])
def test_redistribute_numbering_gloo(world):
    """slab.redistribute after migration: local numbering, computeNodeOffsets and the
    nonlocal nodes with their owners' global indices, against the oracle's
    LDataManager::computeNodeDistribution over the whole level (tests/ldist_check.py)."""
    from ldist_check import check_node_distribution
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_redist_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in res if r[1] != "ok"]
    assert not bad, bad[0][1]
    res.sort(key=lambda r: r[0])
    assert all(r[2] for r in res)
    X_all = np.concatenate([r[4] for r in res])
    lag_all = np.concatenate([r[5] for r in res])
    n_ghost = check_node_distribution([r[3] for r in res], X_all, lag_all, [12, 10, 32], world, 2)
    assert n_ghost > 0
    # ghost_X holds the owners' positions bit for bit (markers just above z = 0 included)
    owner_X = {}
    for r in res:
        for lg, x in zip(r[3]["lag"], r[3]["X"]):
            owner_X[int(lg)] = x
    tiny = 0
    for r in res:
        for lg, x in zip(r[3]["ghost_lag"], r[3]["ghost_X"]):
            assert np.array_equal(x, owner_X[int(lg)]), (r[0], int(lg), x, owner_X[int(lg)])
            tiny += 0.0 < x[2] < 1e-12
    assert tiny > 0


# ---------------------------------------------------------------------------- lazy cadence
def _cadence_worker(rank, world, port, k, nsteps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle as ora
        from ibamr_amd.slab import Slab, migrate, redistribute
        N = [16, 16, 32]
        slab = Slab(N, world, rank, 3)
        slack = slab.ghost - (slab.ghost - 1)  # the ghost width's spare cell (bench.py --regrid-every)
        g = torch.Generator().manual_seed(77)
        M = 3000
        Xg = torch.rand((M, 3), dtype=torch.float64, generator=g) * 0.6 + 0.2  # no periodic wrap in the test
        Xg[:, 2] = torch.rand(M, dtype=torch.float64, generator=g) * 0.4 + 0.3
        lag_g = torch.randperm(M, generator=g).to(torch.int32)
        Fg = torch.rand((M, 3), dtype=torch.float64, generator=g)
        cz = (Xg[:, 2] / slab.dx[2]).floor().long()
        mine = (cz >= slab.z0) & (cz < slab.z1)
        dt = 0.3 * slab.dx[2]

        def vel(X):  # a smooth field moving markers across the interior slab faces
            return torch.stack([torch.zeros_like(X[:, 0]), torch.zeros_like(X[:, 0]),
                                torch.sin(2 * np.pi * X[:, 0]) * torch.cos(2 * np.pi * X[:, 1])], dim=1)

        boxes = [([0, 0, slab.z0], [N[0] - 1, N[1] - 1, slab.z1 - 1])]
        dx = [1.0 / n for n in N]

        def numbering(Xa, la, ghost):
            o, nl, nn = ora.level_node_distribution(Xa.numpy(), la.numpy(), boxes, [0, 0, 0], [n - 1 for n in N],
                                                    [0.0] * 3, dx, ghost)
            return torch.from_numpy(o), nl, nn

        def reorder(order, *arrays):
            return [a[order.long()] for a in arrays]

        def wrap(Xw):
            return Xw

        def run(lazy):
            X, F, lag = Xg[mine].clone(), Fg[mine].clone(), lag_g[mine].clone()
            out, drift_ok = [], True
            for t in range(1, nsteps + 1):
                X = X + dt * vel(X)
                regrid = t % k == 0
                if not lazy or regrid:
                    X, (F, lagf) = migrate(slab, X, [F, lag.to(torch.float64)], cell_order=False)
                    lag = lagf.to(torch.int32)
                else:  # between regrids: the markers keep their rank, within the slack
                    c = (X[:, 2] / slab.dx[2]).floor()
                    drift_ok = drift_ok and bool(((c >= slab.z0 - slack) & (c < slab.z1 + slack)).all())
                if regrid:
                    d = redistribute(slab, None, X, [F], lag, numbering=numbering, reorder=reorder, wrap=wrap)
                    X, F, lag = d.X, d.fields[0], d.lag
                    out.append(d)
            return out, drift_ok

        per_step, _ = run(False)
        lazy, drift_ok = run(True)
        same = len(per_step) == len(lazy) and all(
            torch.equal(a.X, b.X) and torch.equal(a.lag, b.lag) and torch.equal(a.fields[0], b.fields[0])
            and a.offset == b.offset and a.num_nodes == b.num_nodes and torch.equal(a.ghost_X, b.ghost_X)
            and torch.equal(a.ghost_lag, b.ghost_lag) and torch.equal(a.ghost_petsc, b.ghost_petsc)
            for a, b in zip(per_step, lazy))
        moved = sum(int(d.num_nodes) for d in lazy)
        q.put((rank, "ok", same, drift_ok, moved))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc(), False, False, 0))


@pytest.mark.parametrize("world,k", [(2, 3), (4, 3), (2, 1)])
def test_lazy_regrid_cadence_gloo(world, k):
    """The reference's lazy cadence (migrate and renumber every k-th step, markers kept
    on their rank in between, IBHierarchyIntegrator.cpp:495-508): at every regrid step
    the node distribution -- owned positions, fields, Lagrangian indices, offsets,
    nonlocal nodes -- equals, entry by entry, the one of migrating every step; between
    regrids every marker stays within the ghost width's spare cell of its slab."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cadence_worker, args=(r, world, port, k, 3 * k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in res if r[1] != "ok"]
    assert not bad, bad[0][1]
    assert all(r[2] for r in res), "lazy cadence differs from per-step migration at a regrid step"
    assert all(r[3] for r in res), "a marker drifted past the slack between regrids"
