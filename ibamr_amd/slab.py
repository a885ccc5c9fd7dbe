"""Slab decomposition of a uniform periodic grid over GPUs (one process per GPU).

The finest-level Cartesian grid is cut into z-slabs (z is the slowest Fortran
index, so a slab and each of its ghost plane blocks are contiguous).  Rank r owns
cells z in [z0, z1) and the markers whose stencil anchor lies there.  Two
exchange steps per IB step, both point-to-point with the +/-z
neighbours over RCCL (torch.distributed "nccl" = RCCL on ROCm), grouped so each
direction is one send/recv pair per array:

* ``halo_fill`` -- before interpolation: every ghost point gets its periodic
  interior value.  x/y wrap locally (ibtk_le_fill_periodic_ghosts), z ghost
  planes come from the neighbours (the RefineSchedule::fillData of
  LDataManager.cpp:748-751).
* ``ghost_sum`` -- after spreading the rank's own markers into its ghosted slab
  (ghosts zeroed first): z ghost planes are sent to the neighbour that owns them
  and added into its interior planes, then x/y ghosts fold locally.  Every
  destination point receives its sources in a fixed order (own value, then the
  plane from below, then from above, then the x/y folds), so results are
  bit-stable run to run.

For the side-centred z component the face z1 of rank r is face z0 of rank r+1;
each rank treats faces [z0, z1) as its unique interior and z1 as a ghost, so the
upper ghost block of that component is ghost+1 planes thick.

Only ``width`` ghost planes per face are exchanged (Slab.width, default the ghost
width).  A stencil of a marker inside the slab reaches W/2 planes beyond it (IB_4:
2 -- the cell frame's NINT anchor gives ic_lower >= z0 - 2 and ic_upper <= z1 + 1,
the side frame's one plane less below): that many suffice when the markers are
migrated every step; the reference's ghost width W/2 + 1 (getMinimumGhostWidth)
holds the slack for markers that drift up to a cell past the slab between regrids
(CFL_WIDTH, LDataManager.cpp:167), the lazy cadence's case.

The local periodic operations are injectable (``local_fill``/``local_fold``) so
the exchange logic can be tested with gloo on CPU; the product default is the
HIP library, and nothing falls back silently.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import torch


def _rows(f: torch.Tensor) -> torch.Tensor:
    """f as (rows, columns): a rank may hold no markers, and reshape(0, -1) is ambiguous."""
    return f.reshape(f.shape[0], 1) if f.dim() == 1 else f.flatten(1)


@dataclass
class Slab:
    N: Sequence[int]      # global cells per dim
    P: int                # ranks along z
    rank: int
    ghost: int
    L: Sequence[float] = (1.0, 1.0, 1.0)
    align: int = 0        # > 0: the arrays' rows padded to a multiple of `align` (Geometry.aligned)
    width: Optional[int] = None  # ghost planes exchanged per face (None: ghost)

    def __post_init__(self):
        if self.N[2] % self.P:
            raise ValueError(f"N_z={self.N[2]} not divisible by {self.P} ranks")
        if self.width is None:
            self.width = self.ghost
        if not 0 < self.width <= self.ghost:
            raise ValueError(f"exchange width {self.width} outside [1, ghost={self.ghost}]")
        self.nz = self.N[2] // self.P
        if self.P > 1 and self.nz < 2 * self.ghost + 2:
            raise ValueError("slab thinner than 2*ghost+2 planes")
        self.z0 = self.rank * self.nz
        self.z1 = self.z0 + self.nz
        self.dx = [self.L[d] / self.N[d] for d in range(3)]
        self.up = (self.rank + 1) % self.P
        self.down = (self.rank - 1) % self.P

    def geometry(self):
        from .le import Geometry
        g = Geometry([0, 0, self.z0], [self.N[0] - 1, self.N[1] - 1, self.z1 - 1], self.ghost, self.dx,
                     [0.0, 0.0, self.z0 * self.dx[2]],
                     [self.L[0], self.L[1], self.z1 * self.dx[2]])
        return g.aligned(self.align) if self.align else g

    # plane blocks of one side component array (leading dim = z planes): the `width`
    # ghost planes next to each face and the interior planes they mirror
    def blocks(self, comp: int):
        g, nz, w = self.ghost, self.nz, self.width
        up = w + (1 if comp == 2 else 0)   # upper ghost thickness (z-faces carry z1)
        return {
            "lo_ghost": (g - w, g),               # -> down neighbour's top interior
            "hi_ghost": (g + nz, g + nz + up),    # -> up neighbour's bottom interior
            "top_int": (g + nz - w, g + nz),      # <- up neighbour's lo_ghost
            "bot_int": (g, g + up),               # <- down neighbour's hi_ghost
        }


class SlabExchange:
    """z-halo fill and ghost-region sum of side-centred arrays across ranks."""

    def __init__(self, slab: Slab, arrays: List[torch.Tensor], ctx=None, group=None,
                 local_fill: Optional[Callable] = None, local_fold: Optional[Callable] = None):
        self.slab = slab
        self.arrays = arrays
        self.group = group
        self.ctx = ctx
        self.geom = slab.geometry()
        self._local_fill = local_fill
        self._local_fold = local_fold
        self.bufs = []
        for c, a in enumerate(arrays):
            b = slab.blocks(c)
            lo0, lo1 = b["lo_ghost"]
            hi0, hi1 = b["hi_ghost"]
            self.bufs.append((torch.empty_like(a[lo0:lo1]), torch.empty_like(a[hi0:hi1])))

    # -- local periodic pieces -------------------------------------------------
    def local_fill(self, periodic):
        if self._local_fill is not None:
            return self._local_fill(self.arrays, periodic)
        from . import le
        le.fill_periodic_ghosts(self.ctx, self.geom, "side", self.arrays, periodic=periodic)

    def local_fold(self, periodic):
        if self._local_fold is not None:
            return self._local_fold(self.arrays, periodic)
        from . import le
        le.fold_periodic_ghosts(self.ctx, self.geom, "side", self.arrays, periodic=periodic)

    # -- exchanges -------------------------------------------------------------------
    def _p2p_start(self, sends, recvs):
        import torch.distributed as dist
        # gloo moves host memory only: device tensors are staged through the host
        # (the multi-rank rehearsal on one GPU; RCCL sends device memory directly)
        stage = dist.get_backend(self.group) == "gloo"
        # plane blocks of pitched arrays (padded rows) are not contiguous: they are
        # packed into / unpacked from contiguous buffers around the transfer
        ops, back = [], []
        for t, peer in sends:
            if stage and t.is_cuda:
                t = t.cpu()
            elif not t.is_contiguous():
                t = t.contiguous()
            ops.append(dist.P2POp(dist.isend, t, peer, group=self.group))
        for t, peer in recvs:
            if stage and t.is_cuda:
                h = torch.empty(t.shape, dtype=t.dtype)
                back.append((h, t))
                t = h
            elif not t.is_contiguous():
                h = torch.empty(t.shape, dtype=t.dtype, device=t.device)
                back.append((h, t))
                t = h
            ops.append(dist.P2POp(dist.irecv, t, peer, group=self.group))
        # RCCL: the transfers run on the communicator's stream, ordered after the
        # work already queued on the current stream; what is queued next overlaps
        return (dist.batch_isend_irecv(ops) if ops else []), back

    @staticmethod
    def _p2p_wait(handle):
        works, back = handle
        for w in works:
            w.wait()  # RCCL: the current stream waits for the transfers (no host block)
        for h, t in back:
            t.copy_(h)

    def _p2p(self, sends, recvs):
        self._p2p_wait(self._p2p_start(sends, recvs))

    def _windowed(self, work, mode):
        """work() restricted to the sweep items inside (1) / outside (2) the rank's
        own planes [z0, z1) (ibtk_le_ctx_set_plane_window); the two halves add up to
        one unrestricted call bit for bit.  The context's previous window (and with it
        the item cutting of later binnings) is restored afterwards."""
        s = self.slab
        prev = getattr(self.ctx, "plane_window", (0, 0, -1))
        self.ctx.set_plane_window(mode, s.z0, s.z1 - 1)
        try:
            work()
        finally:
            self.ctx.set_plane_window(*prev)

    def cut_items(self):
        """Make the markers binned from now on on this context cut their sweep items
        at the slab faces (ibtk_le_ctx_set_plane_window with mode 0), so the
        boundary items of an overlapped call are only the few planes next to a face."""
        if self.slab.P > 1 and self.ctx is not None:
            self.ctx.set_plane_window(0, self.slab.z0, self.slab.z1 - 1)

    def halo_fill(self, work=None, local: bool = True):
        """Every ghost point := its periodic interior value (before interpolation).

        work: optional callable (the interpolation); it then runs in two halves,
        the sweep items that read only the rank's own planes while the z planes
        are in flight, and the items next to the slab faces after they land.
        local=False: no local x/y (one rank: x/y/z) periodic fill -- the work reads
        those ghosts at their periodic images itself (ibtk_le_fill_interp); only the z
        planes from the neighbours are exchanged."""
        s = self.slab
        if s.P == 1:
            if local:
                self.local_fill([1, 1, 1])
            if work is not None:
                work()
            return
        if local:
            self.local_fill([1, 1, 0])   # x/y ghosts of the interior planes
        sends, recvs = [], []
        for c, a in enumerate(self.arrays):
            b = s.blocks(c)
            t0, t1 = b["top_int"]
            b0, b1 = b["bot_int"]
            lo0, lo1 = b["lo_ghost"]
            hi0, hi1 = b["hi_ghost"]
            # RCCL matches a peer's sends and receives in issue order and ignores
            # tags, so every exchange posts its receives from a peer in the order
            # that peer posts the matching sends (with P = 2, up == down), and
            # uses one tag, so gloo matches the same way
            sends.append((a[t0:t1], s.up))      # my top planes -> up's lower ghosts
            sends.append((a[b0:b1], s.down))    # my bottom planes -> down's upper ghosts
            recvs.append((a[lo0:lo1], s.down))  # down's top planes (its first send)
            recvs.append((a[hi0:hi1], s.up))    # up's bottom planes (its second send)
        h = self._p2p_start(sends, recvs)
        if work is not None:
            self._windowed(work, 1)
        self._p2p_wait(h)
        if work is not None:
            self._windowed(work, 2)

    def ghost_sum(self, work=None):
        """Fold every ghost value onto its owner's interior point (after spreading).

        work: optional callable (the spreading into the zeroed-ghost arrays); it
        then runs in two halves, the sweep items owning planes next to the slab
        faces first, and the interior items while the ghost planes are in flight."""
        s = self.slab
        if s.P == 1:
            if work is not None:
                work()
            return self.local_fold([1, 1, 1])
        if work is not None:
            self._windowed(work, 2)
        sends, recvs = [], []
        for c, a in enumerate(self.arrays):
            b = s.blocks(c)
            lo0, lo1 = b["lo_ghost"]
            hi0, hi1 = b["hi_ghost"]
            rlo, rhi = self.bufs[c]
            sends.append((a[lo0:lo1], s.down))  # first send
            sends.append((a[hi0:hi1], s.up))    # second send
            # receives in the peers' send order: up's lower ghosts (its first send,
            # they land on my top planes), then down's upper ghosts (its second
            # send, my bottom planes)
            recvs.append((rlo, s.up))
            recvs.append((rhi, s.down))
        h = self._p2p_start(sends, recvs)
        if work is not None:
            self._windowed(work, 1)
        self._p2p_wait(h)
        for c, a in enumerate(self.arrays):
            b = s.blocks(c)
            rlo, rhi = self.bufs[c]
            b0, b1 = b["bot_int"]
            t0, t1 = b["top_int"]
            a[b0:b1].add_(rhi)   # from below first ...
            a[t0:t1].add_(rlo)   # ... then from above
        self.local_fold([1, 1, 0])


class GhostMarkers:
    """The reference's spread exchange: ghost markers instead of a grid reduction.

    LDataManager::spread (LDataManager.cpp:555-675) spreads, per patch, the list of
    every marker whose stencil can reach the patch -- its own and the ghost nodes a
    neighbouring rank owns (LData ghost nodes, kept current by
    LData::beginGhostUpdate) -- into the patch's ghosted data, and keeps the
    interior: no ghost-region sum.  Here a rank sends the markers (position and
    force) whose cell lies within ``ghost`` planes of a slab face to the
    neighbour across it; each rank spreads its own plus the received markers and
    keeps its own planes (the z ghost planes are left as they fall), then folds
    x/y locally.  Markers crossing the periodic z wrap arrive shifted by -+L_z
    (the periodic_shift of LIndexSetData's ghost lists).  One pair of
    point-to-point messages per direction and step (the counts, then the data),
    SURVEY.md 8(e) "reference mode": ~2 ghost/N_z of the markers move instead of
    3 x ghost planes of grid per face.  Results match the grid-sum mode and one
    rank within the spread tolerance, and are bit-stable run to run.
    """

    def __init__(self, slab: Slab, group=None, width: Optional[int] = None):
        self.slab = slab
        self.group = group
        # planes of markers sent per face: the stencils' reach (Slab.width) for the
        # spread; the full ghost width for redistribute's nonlocal nodes (the ghost box)
        self.width = slab.width if width is None else width

    def _p2p(self, sends, recvs):
        import torch.distributed as dist
        stage = dist.get_backend(self.group) == "gloo"
        ops, back = [], []
        for t, peer in sends:
            ops.append(dist.P2POp(dist.isend, t.cpu() if stage and t.is_cuda else t, peer, group=self.group))
        for t, peer in recvs:
            if stage and t.is_cuda:
                h = torch.empty(t.shape, dtype=t.dtype)
                back.append((h, t))
                t = h
            ops.append(dist.P2POp(dist.irecv, t, peer, group=self.group))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        for h, t in back:
            t.copy_(h)

    def select(self, X: torch.Tensor):
        """(to_up, to_down): indices of the markers within `width` cells of the
        upper / lower slab face (a marker can be in both when the slab is thin)."""
        s = self.slab
        cz = torch.clamp((X[:, 2] / s.dx[2]).floor().long(), 0, s.N[2] - 1)
        up = (cz >= s.z1 - self.width).nonzero().squeeze(1)
        down = (cz < s.z0 + self.width).nonzero().squeeze(1)
        return up, down

    def exchange(self, X: torch.Tensor, F: torch.Tensor):
        """Own markers followed by the ghost markers from below, then from above:
        (X_all, F_all, n_own).  X: (M, 3), F: (M, d) float64 of this rank."""
        s = self.slab
        if s.P == 1:
            return X, F, X.shape[0]
        up, down = self.select(X)
        data = torch.cat([X, _rows(F).to(X.dtype)], dim=1)
        send_up, send_down = data[up].contiguous(), data[down].contiguous()
        # counts, then data; each peer's receives in the order it sends (RCCL
        # matches a pair's messages in issue order; with P = 2 up == down):
        # sends [to up, to down], receives [from down (its "to up"), from up]
        dev = X.device
        cu = torch.tensor([send_up.shape[0]], dtype=torch.int64, device=dev)
        cd = torch.tensor([send_down.shape[0]], dtype=torch.int64, device=dev)
        rd, ru = torch.empty_like(cu), torch.empty_like(cd)
        self._p2p([(cu, s.up), (cd, s.down)], [(rd, s.down), (ru, s.up)])
        nd, nu = (int(v) for v in torch.cat([rd, ru]).cpu().tolist())  # the step's one host sync
        D = data.shape[1]
        from_down = torch.empty((nd, D), dtype=data.dtype, device=dev)
        from_up = torch.empty((nu, D), dtype=data.dtype, device=dev)
        sends = [(t, peer) for t, peer in ((send_up, s.up), (send_down, s.down))]
        recvs = [(t, peer) for t, peer in ((from_down, s.down), (from_up, s.up))]
        self._p2p(sends, recvs)
        Lz = s.L[2]
        if s.rank == 0 and nd:
            from_down[:, 2] -= Lz   # rank P-1's top planes sit below z = 0
        if s.rank == s.P - 1 and nu:
            from_up[:, 2] += Lz     # rank 0's bottom planes sit above z = L_z
        allm = torch.cat([data, from_down, from_up], dim=0)
        Xa = allm[:, :3].contiguous()
        Fa = allm[:, 3:].reshape((allm.shape[0],) + tuple(F.shape[1:])).to(F.dtype).contiguous()
        return Xa, Fa, X.shape[0]


def update_and_migrate(slab: Slab, ctx, scheme: str, dt: float, X: torch.Tensor, U0: torch.Tensor,
                       fields: Sequence[torch.Tensor] = (), U1: Optional[torch.Tensor] = None, group=None):
    """Position update and migration on the device (IBMethod's eulerStep/midpointStep/
    trapezoidalStep, IBMethod.cpp:619-681, then the redistribution of
    LDataManager.cpp:1504-1959 each step).

    One fused HIP pass updates, wraps and classifies the markers and partitions them
    stably (ibtk_le_slab_update_partition: [stay | down | up | further]); the leavers go
    to the z-neighbours with two point-to-point messages each way (the counts, then the
    rows).  A step moves markers by less than a slab, so "further" is empty; if a rank
    finds it is not, every rank takes the all-to-all path of ``migrate`` (one max-reduce
    of the flag decides, together with the counts).  The host syncs once, for the count
    vector the receive buffers need.  Returns (X, fields): the stayers in their order,
    then the arrivals from below, then from above (``migrate(cell_order=False)``'s
    contract with a neighbour order)."""
    import torch.distributed as dist
    from . import le
    M = X.shape[0]
    Xn, order, counts = le.slab_update_partition(ctx, scheme, dt, X, U0, slab.L, slab.N[2], slab.P, slab.rank,
                                                 U1=U1)
    flat = [_rows(f) for f in fields]
    if slab.P == 1:
        return Xn, list(fields)  # everything stays; the order is the input order
    # counts to the neighbours and the global "further" flag
    send_c = torch.stack([counts[1], counts[2]]).to(torch.int64)
    far = counts[3:4].to(torch.int64).clone()
    rc_down, rc_up = torch.empty(1, dtype=torch.int64, device=X.device), torch.empty(1, dtype=torch.int64,
                                                                                    device=X.device)
    gm = GhostMarkers(slab, group)
    gm._p2p([(send_c[1:2], slab.up), (send_c[0:1], slab.down)], [(rc_down, slab.down), (rc_up, slab.up)])
    dist.all_reduce(far, op=dist.ReduceOp.MAX, group=group)
    host = torch.cat([counts.to(torch.int64), rc_down, rc_up, far]).cpu().tolist()  # the one host sync
    n_stay, n_down, n_up, _, r_down, r_up, any_far = host
    if any_far:
        return migrate(slab, Xn, list(fields), group=group, cell_order=False)
    data = torch.cat([Xn] + [f.to(Xn.dtype) for f in flat], dim=1)
    stay = data[order[:n_stay].long()]
    to_down = data[order[n_stay:n_stay + n_down].long()].contiguous()
    to_up = data[order[n_stay + n_down:n_stay + n_down + n_up].long()].contiguous()
    D = data.shape[1]
    from_down = torch.empty((r_down, D), dtype=data.dtype, device=data.device)
    from_up = torch.empty((r_up, D), dtype=data.dtype, device=data.device)
    # each peer's receives in the order it sends (P = 2: up == down)
    gm._p2p([(to_up, slab.up), (to_down, slab.down)], [(from_down, slab.down), (from_up, slab.up)])
    allm = torch.cat([stay, from_down, from_up], dim=0)
    Xo = allm[:, :3].contiguous()
    outs, k = [], 3
    for f, fl in zip(fields, flat):
        w = fl.shape[1]
        outs.append(allm[:, k:k + w].reshape((allm.shape[0],) + tuple(f.shape[1:])).to(f.dtype).contiguous())
        k += w
    return Xo, outs


def update_and_migrate_fixed(slab: Slab, ctx, scheme: str, dt: float, X: torch.Tensor, U0: torch.Tensor,
                             fields: Sequence[torch.Tensor], n_dev: torch.Tensor, send_cap: int,
                             U1: Optional[torch.Tensor] = None, group=None):
    """``update_and_migrate`` without a host sync: fixed-capacity arrays whose row count
    lives on the device.

    X, U0 (U1) and the fields hold ``capacity`` rows of which the first n_dev[0] (a
    device int32) are markers.  The fused update + partition runs over those rows
    (ibtk_le_slab_update_partition_count); the leavers are packed into send buffers of
    ``send_cap`` rows per neighbour (ibtk_le_slab_migrate_pack) and exchanged at that
    fixed size together with their counts -- nothing the host must read before posting
    the receives; the stayers (in order), then the arrivals from below, then from above
    are unpacked into new capacity-sized arrays (ibtk_le_slab_migrate_unpack).  Returns
    (X, fields, n_dev), ready for ``Markers.bin_count``.  Leavers beyond send_cap, a
    marker moving further than one slab, or arrivals beyond the capacity raise device
    flag 8 at the next ``ctx.synchronize()`` (never a silent drop).  Bitwise the same
    rows, in the same order, as ``update_and_migrate``."""
    from . import le
    C = X.shape[0]
    Xn, order, counts = le.slab_update_partition_count(ctx, scheme, dt, X, U0, slab.L, slab.N[2], slab.P, slab.rank,
                                                       n_dev, U1=U1)
    flat = [_rows(f) for f in fields]
    data = torch.cat([Xn] + [f.to(Xn.dtype) for f in flat], dim=1).contiguous()
    D = data.shape[1]
    if slab.P == 1:
        n_out = counts[0:1].clone()
        outs, k = [], 3
        for f, fl in zip(fields, flat):
            w = fl.shape[1]
            outs.append(data[:, k:k + w].reshape(f.shape).to(f.dtype).contiguous())
            k += w
        return Xn, outs, n_out
    send_down = torch.empty((send_cap, D), dtype=data.dtype, device=data.device)
    send_up = torch.empty_like(send_down)
    le.slab_migrate_pack(ctx, data, order, counts, send_down, send_up)
    gm = GhostMarkers(slab, group)
    rc = torch.empty(2, dtype=torch.int32, device=X.device)  # [from below, from above]
    # each peer's receives in the order it sends (P = 2: up == down): counts, then rows
    gm._p2p([(counts[2:3], slab.up), (counts[1:2], slab.down)], [(rc[0:1], slab.down), (rc[1:2], slab.up)])
    from_down = torch.empty_like(send_down)
    from_up = torch.empty_like(send_down)
    gm._p2p([(send_up, slab.up), (send_down, slab.down)], [(from_down, slab.down), (from_up, slab.up)])
    out = torch.empty((C, D), dtype=data.dtype, device=data.device)
    n_out = torch.empty(1, dtype=torch.int32, device=X.device)
    le.slab_migrate_unpack(ctx, data, order, counts, rc, from_down, from_up, out, n_out)
    Xo = out[:, :3].contiguous()
    outs, k = [], 3
    for f, fl in zip(fields, flat):
        w = fl.shape[1]
        outs.append(out[:, k:k + w].reshape((C,) + tuple(f.shape[1:])).to(f.dtype).contiguous())
        k += w
    return Xo, outs, n_out


def migrate(slab: Slab, X: torch.Tensor, fields: Sequence[torch.Tensor] = (), group=None, cell_order: bool = True):
    """Move every marker to the rank whose slab holds its cell, after a position update.

    The reference migrates at regrid (LDataManager::beginDataRedistribution /
    endDataRedistribution, LDataManager.cpp:1337-1959, owner by
    IndexUtilities::getCellIndex); SURVEY.md 8(e) asks for it after every update.
    One all-to-all of counts and one of data (torch.distributed: RCCL on GPUs,
    gloo on CPU).  Positions are wrapped into the periodic box [0, L)^3 first.

    X: (M, 3) float64; fields: tensors with M rows (any trailing shape, cast to
    float64 for the exchange and back).  Returns (X, fields) of the markers this
    rank owns afterwards.  With cell_order they are stably sorted by cell (z, y, x),
    the local numbering LDataManager::computeNodeDistribution gives
    (LDataManager.cpp:2839-3027).  Without it only the leavers move: the markers
    that stay keep their order and the arrivals follow in source-rank order.  That
    is the cheap per-step form, since after a small position update few markers
    cross a slab face.  Deterministic either way: the same inputs give the same
    order on every run.
    """
    import torch.distributed as dist
    M = X.shape[0]
    L = torch.tensor(list(slab.L), dtype=X.dtype, device=X.device)
    Xw = torch.remainder(X, L)
    Xw = torch.where(Xw >= L, Xw - L, Xw)  # remainder can round up to L
    cell = [torch.clamp((Xw[:, d] / slab.dx[d]).floor().long(), 0, slab.N[d] - 1) for d in range(3)]
    dest = cell[2] // slab.nz
    cols = [Xw] + [_rows(f).to(X.dtype) for f in fields]
    widths = [c.shape[1] for c in cols]
    data = torch.cat(cols, dim=1)
    stay = None
    if not cell_order:  # keep the stayers in place, send only the leavers
        keep = dest == slab.rank
        stay = data[keep]
        go = (~keep).nonzero().squeeze(1)
        dest = dest[go]
        data = data[go]
    order = torch.argsort(dest, stable=True)
    send = data[order].contiguous()
    send_counts = torch.bincount(dest, minlength=slab.P).to(torch.int64)
    if slab.P == 1:
        recv = send
    else:
        # gloo moves host memory only (the one-GPU rehearsal): stage through the host
        host = dist.get_backend(group) == "gloo" and send.is_cuda
        sc = send_counts.cpu() if host else send_counts
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=group)
        # the split sizes must be host integers (all_to_all_single's signature):
        # one device->host copy of both count vectors, the step's only host sync
        counts = torch.stack([sc, rc]).cpu().tolist() if not host else [sc.tolist(), rc.tolist()]
        D = send.shape[1]
        sd = send.cpu() if host else send
        recv = torch.empty((sum(counts[1]), D), dtype=send.dtype, device=sd.device)
        dist.all_to_all_single(recv, sd, output_split_sizes=counts[1], input_split_sizes=counts[0], group=group)
        recv = recv.to(send.device)
    if stay is not None:
        recv = torch.cat([stay, recv], dim=0)
    if cell_order and recv.shape[0]:
        c = [torch.clamp((recv[:, d] / slab.dx[d]).floor().long(), 0, slab.N[d] - 1) for d in range(3)]
        key = (c[2] * slab.N[1] + c[1]) * slab.N[0] + c[0]
        recv = recv[torch.argsort(key, stable=True)]
    outs, k = [], 0
    for w in widths:
        outs.append(recv[:, k:k + w])
        k += w
    Xn = outs[0].contiguous()
    fn = [o.reshape((o.shape[0],) + tuple(f.shape[1:])).to(f.dtype).contiguous() for o, f in zip(outs[1:], fields)]
    return Xn, fn


@dataclass
class NodeDistribution:
    """A rank's nodes after ``redistribute`` (LDataManager's per-level state after
    endDataRedistribution): the owned nodes in local order -- global (PETSc) index
    ``offset + i`` for row i -- and the nonlocal (ghost) nodes in the reference's
    nonlocal order with the global index their owner gave them."""
    X: torch.Tensor
    fields: List[torch.Tensor]
    lag: torch.Tensor             # int32 Lagrangian index of each owned node
    order: torch.Tensor           # owned row i was input row order[i]
    offset: int                   # computeNodeOffsets: first global index of this rank
    num_nodes: int                # computeNodeOffsets: nodes of the whole level
    ghost_X: torch.Tensor
    ghost_lag: torch.Tensor       # int32
    ghost_petsc: torch.Tensor     # int64 global index of each nonlocal node


def redistribute(slab: Slab, ctx, X: torch.Tensor, fields: Sequence[torch.Tensor], lag: torch.Tensor,
                 group=None, numbering: Optional[Callable] = None, reorder: Optional[Callable] = None,
                 wrap: Optional[Callable] = None):
    """Number a rank's markers the way LDataManager does at redistribution, across ranks.

    After ``migrate``/``update_and_migrate`` every marker sits on the rank whose slab
    (the rank's one patch of the level) holds its cell.  Positions are wrapped into the
    periodic box first (beginDataRedistribution, LDataManager.cpp:1385-1399).  Then, as
    LDataManager::computeNodeDistribution (LDataManager.cpp:2839-3027):

    * local numbering -- the owned markers in the slab's cell order (x fastest),
      Lagrangian order within a cell, repeated (cell, Lagrangian index) pairs kept
      once (ibtk_le_level_node_distribution), and the LData arrays reordered into it
      (ibtk_le_ldata_reorder; endDataRedistribution's VecScatter,
      LDataManager.cpp:1823-1917, for the rows that stayed on this rank);
    * computeNodeOffsets (LDataManager.cpp:3029-3047) -- one all-gather of the local
      counts; node i of rank r has global index offset_r + i;
    * nonlocal nodes -- the neighbours' markers within ``ghost`` cells of the slab
      faces (GhostMarkers' exchange, which carries each one's Lagrangian and global
      index, so no AO lookup is needed: AOApplicationToPetsc at :2995-3000 maps the
      Lagrangian index to the global index its owner assigned), numbered after the
      local nodes in the ghost-box walk order; ``ghost_X`` holds the owners'
      positions (in [0, L)), as the reference's ghosted LData does.

    ``numbering(X, lag, ghost) -> (order, n_local, n_nonlocal)``,
    ``reorder(order, *arrays) -> [arrays]`` and ``wrap(X) -> X`` are injectable so the
    rank logic runs on CPU with gloo (tests); the product default is the HIP library
    (ibtk_le_level_node_distribution, ibtk_le_ldata_reorder, ibtk_le_wrap_positions)."""
    import torch.distributed as dist
    from . import le
    if lag.dtype != torch.int32 or lag.numel() != X.shape[0]:
        raise ValueError("lag: one int32 Lagrangian index per marker")
    if numbering is None:
        geoms = [slab.geometry()]
        dom_hi = [n - 1 for n in slab.N]

        def numbering(Xa, la, ghost):
            return le.level_node_distribution(ctx, geoms, [0, 0, 0], dom_hi, Xa, ghost, lag=la)
    if reorder is None:
        def reorder(order, *arrays):
            return le.ldata_reorder(ctx, order, *arrays)
    # beginDataRedistribution's wrap into the periodic domain (LDataManager.cpp:1385-1399)
    if wrap is None:
        def wrap(Xw):
            return le.wrap_positions(ctx, Xw, [0.0, 0.0, 0.0], list(slab.L))
    X = wrap(X.contiguous().clone())
    order, nl, nn = numbering(X, lag, 0)
    if nn:
        raise RuntimeError(f"rank {slab.rank}: {nn} markers outside the slab; migrate before redistribute")
    M = X.shape[0]
    flat = [_rows(f).to(X.dtype).contiguous() for f in fields]
    Xn, *fn = reorder(order, X, *flat) if nl else [X[:0]] + [f[:0] for f in flat]
    fn = [o.reshape((o.shape[0],) + tuple(f.shape[1:])).to(f.dtype).contiguous() for o, f in zip(fn, fields)]
    lagn = lag[order.long()]
    # computeNodeOffsets: the local counts of every rank
    counts = [nl]
    if slab.P > 1:
        host = dist.get_backend(group) == "gloo"
        c = torch.tensor([nl], dtype=torch.int64, device="cpu" if host else X.device)
        allc = [torch.empty_like(c) for _ in range(slab.P)]
        dist.all_gather(allc, c, group=group)
        counts = [int(v) for v in torch.cat(allc).cpu().tolist()]
    offset = sum(counts[:slab.rank])
    num_nodes = sum(counts)
    # nonlocal nodes: the neighbours' markers near the slab faces, with their indices
    # and their owners' z (the exchange shifts the markers that cross the periodic z wrap
    # by -+L_z, and z + L_z - L_z need not give z back: the owner's bits travel along)
    ids = torch.stack([lagn.to(X.dtype), offset + torch.arange(nl, dtype=X.dtype, device=X.device), Xn[:, 2]],
                      dim=1)
    Xa, Ia, n_own = GhostMarkers(slab, group, width=slab.ghost).exchange(Xn, ids)
    gX = Xa[:0]
    gI = Ia[:0]
    if Xa.shape[0] > n_own:
        Xg = Xa[n_own:].clone()
        Ig = Ia[n_own:]
        Xg[:, 2] = Ig[:, 2]  # the owners' positions, bit for bit
        # the nonlocal order depends only on the nonlocal markers (their cells, images and
        # Lagrangian indices), so only they are numbered here: every one lies outside the
        # slab's box, so all of them come out nonlocal
        order2, nl2, nn2 = numbering(Xg.contiguous(), Ig[:, 0].to(torch.int32).contiguous(), slab.ghost)
        if nl2 != 0:
            raise RuntimeError(f"rank {slab.rank}: {nl2} received ghost markers inside the slab")
        sel = order2[:nn2].long()
        gX, gI = Xg[sel].contiguous(), Ig[sel]
    return NodeDistribution(Xn, fn, lagn, order, offset, num_nodes, gX, gI[:, 0].to(torch.int32),
                            gI[:, 1].to(torch.int64))
