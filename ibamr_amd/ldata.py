"""LDataManager's two coupling entry points for one uniform patch on one GPU.

Mirrors ``IBTK::LDataManager::spread`` (LDataManager.cpp:555-675, density-weighted
overload :398-470) and ``LDataManager::interp`` (:705-819) for the finest level of
a uniform grid held as one patch per GPU, over the device C-ABI (``le``):

* ``spread(f, F, X)``: copy f, zero it including ghosts, spread the markers over
  the ghost box, fold the ghosts back -- periodic dims by the periodic fold
  (the reference spreads periodic ghost markers instead; same sum, another
  order), then the physical faces by ``accumulateFromPhysicalBoundaryData``
  (:655-659); the duplicated upper faces of periodic axes take their lower
  faces' sums -- and add the copy back on the interior (``f_data_ops->add``,
  :664-665, interior only).
* ``interp(f, F, X)``: fill the ghosts -- physical faces by
  ``setPhysicalBoundaryConditions``, then the periodic dims (the ghost-fill
  schedule, :748-751) -- and interpolate at every marker.
  ``zeroInactivatedComponents`` (:812-815) has no counterpart: markers here have
  no inactivation flag.

The markers are binned once per position update (``bin``), as
``beginDataRedistribution`` / ``endDataRedistribution`` re-bin them
(LDataManager.cpp:1337-1959); side-centred data only (``sc_data``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

from . import le


@dataclass
class RobinBc:
    """Constant Robin coefficients a u + b du/dn = g per (component axis, face)
    (RobinBcCoefStrategy::setBcCoefs on a constant box); faces 2 d + upper."""

    physical: Sequence[int]
    a: object = 1.0
    b: object = 0.0
    g: object = 0.0


@dataclass
class LDataLevel:
    ctx: le.Context
    geom: le.Geometry
    kernel: str = "IB_4"
    periodic: Sequence[int] = (1, 1, 1)
    bc: Optional[RobinBc] = None
    _bins: Optional[le.Markers] = field(default=None, init=False, repr=False)
    _old: Optional[list] = field(default=None, init=False, repr=False)

    def __post_init__(self):
        nd = self.geom.ndim
        self.periodic = [int(bool(p)) for p in list(self.periodic)[:nd]]
        if self.bc is not None:
            for d in range(nd):
                if self.periodic[d] and (self.bc.physical[2 * d] or self.bc.physical[2 * d + 1]):
                    raise ValueError(f"dim {d} is periodic and has a physical face")

    def bin(self, X: torch.Tensor):
        """Re-bin the markers after a position update (device radix sort)."""
        if self._bins is None:
            self._bins = le.Markers(self.ctx)
        self._bins.bin(self.geom, self.kernel, X)
        return self

    def _interior(self, a: int, t: torch.Tensor) -> torch.Tensor:
        g = self.geom.gcw
        nd = self.geom.ndim
        sl = []
        for d in reversed(range(nd)):  # torch dims: slowest first
            n = self.geom.iupper[d] - self.geom.ilower[d] + 1 + (1 if d == a else 0)
            sl.append(slice(g[d], g[d] + n))
        return t[tuple(sl)]

    def spread(self, f: Sequence[torch.Tensor], F: torch.Tensor, X: torch.Tensor,
               ds: Optional[torch.Tensor] = None):
        """f += S F (folded), LDataManager::spread (LDataManager.cpp:555-675)."""
        if self._bins is None:
            raise RuntimeError("bin() the markers first")
        # swapData with the cloned index (:590-592): the copy lives in scratch
        # arrays allocated once per level, not per call
        if self._old is None or any(o.shape != t.shape or o.device != t.device for o, t in zip(self._old, f)):
            self._old = [torch.empty_like(t) for t in f]
        old = self._old
        for o, t in zip(old, f):
            o.copy_(t)
        for t in f:
            t.zero_()  # setToScalar(0, interior_only=false) (:593)
        le.spread(self.ctx, self._bins, self.kernel, "side", self.geom, f, F, X, ds=ds)
        if any(self.periodic):
            le.fold_periodic_ghosts(self.ctx, self.geom, "side", f, periodic=self.periodic)
        if self.bc is not None and any(self.bc.physical):
            le.phys_bdry_side(self.ctx, self.geom, f, self.bc.physical, self.bc.a, self.bc.b, self.bc.g,
                              adjoint=True)
        if any(self.periodic):
            # the upper face of a side array along a periodic axis is its lower
            # face's image: both carry the folded sum, as the reference computes
            # both from the same (ghost) markers
            le.fill_periodic_ghosts(self.ctx, self.geom, "side", f, periodic=self.periodic)
        for a, (t, o) in enumerate(zip(f, old)):
            self._interior(a, t).add_(self._interior(a, o))  # f_data_ops->add (:664-665)
        return f

    def interp(self, f: Sequence[torch.Tensor], F: torch.Tensor, X: torch.Tensor):
        """F = J f at every marker, LDataManager::interp (LDataManager.cpp:705-819)."""
        if self._bins is None:
            raise RuntimeError("bin() the markers first")
        if self.bc is not None and any(self.bc.physical):
            le.phys_bdry_side(self.ctx, self.geom, f, self.bc.physical, self.bc.a, self.bc.b, self.bc.g,
                              adjoint=False)
        if any(self.periodic):
            le.fill_periodic_ghosts(self.ctx, self.geom, "side", f, periodic=self.periodic)
        le.interp(self.ctx, self._bins, self.kernel, "side", self.geom, f, F, X)
        return F
