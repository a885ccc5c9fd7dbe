"""Diagnostic: the level interp of cell data, unfused and fused."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from ibamr_amd import le
from oracle import oracle as ora
import test_gpu_level as T

ctx = le.Context(0)
N, P, kernel = 96, 2, "IB_4"
g = ora.min_ghost_width(kernel)
geoms = T._patches(le, N, P, g)
rng = np.random.default_rng(1)
M = 3000
X = rng.uniform(0, 1, (M, 3))
Xd = torch.from_numpy(X).cuda()
lists_i = [(torch.from_numpy(T._lists(geom, X, N, g)[0]).cuda(), None) for geom in geoms]
lvl = le.Level(ctx, geoms, kernel, Xd, lists_i)
for alloc in ("level", "separate"):
    arr = le.alloc_level(geoms, "cell") if alloc == "level" else [geom.alloc("cell") for geom in geoms]
    print(alloc, "shape", tuple(arr[0][0].shape), "array_shape", geoms[0].array_shape("cell", 0, 1))
    for per in arr:
        per[0].uniform_(-1, 1)
    for fused in (False, True):
        Q = torch.full((M, 1), np.nan, dtype=torch.float64, device="cuda")
        if fused:
            lvl.fill_interp("cell", arr, Q, Xd, Q_depth=1)
        else:
            lvl.fill_ghosts("cell", arr)
            lvl.interp("cell", arr, Q, Xd, Q_depth=1)
        ctx.synchronize()
        q = Q.cpu().numpy()
        print(alloc, "fused" if fused else "unfused", "NaN", int(np.isnan(q).sum()), "of", M, q[:3, 0])
