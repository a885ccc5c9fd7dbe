"""Diagnostic: which markers read a NaN in the fused level fill-interp (one case)."""
import sys, itertools
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from ibamr_amd import le
from oracle import oracle as ora
import test_gpu_level as T

kernel, P, centering = "IB_4", 2, "side"
ctx = le.Context(0)
def run(periodic):
    
    N = 48
    g = ora.min_ghost_width(kernel)
    geoms = T._patches(le, N, P, g)
    rng = np.random.default_rng(9)
    M = 30000
    X = rng.uniform(0, 1, (M, 3))
    Xd = torch.from_numpy(X).cuda()
    lists_i = [(torch.from_numpy(T._lists(geom, X, N, g)[0]).cuda(), None) for geom in geoms]
    lvl = le.Level(ctx, geoms, kernel, Xd, lists_i)
    arr = le.alloc_level(geoms, centering)
    n = N // P
    for q, geom in enumerate(geoms):
        tile = [(geom.ilower[d] // n) for d in range(3)]
        for a in range(3):
            v = rng.uniform(-1, 1, tuple(arr[q][a].shape))
            shp = v.shape
            idx = [np.arange(shp[2 - d]) + geom.ilower[d] - g for d in range(3)]
            dirs = [np.where(idx[d] < geom.ilower[d], -1, np.where(idx[d] >= geom.ilower[d] + n, 1, 0)) for d in range(3)]
            ok = [np.where(dirs[d] == 0, True, bool(periodic[d]) | ((tile[d] + dirs[d] >= 0) & (tile[d] + dirs[d] < P))) for d in range(3)]
            ghost = (dirs[2][:, None, None] != 0) | (dirs[1][None, :, None] != 0) | (dirs[0][None, None, :] != 0)
            supplied = ok[2][:, None, None] & ok[1][None, :, None] & ok[0][None, None, :]
            v[ghost & supplied] = np.nan
            arr[q][a].copy_(torch.from_numpy(v))
    Q = torch.full((M, 3), np.nan, dtype=torch.float64, device="cuda")
    lvl.fill_interp(centering, arr, Q, Xd, periodic=list(periodic))
    ctx.synchronize()
    Qh = Q.cpu().numpy()
    bad = np.isnan(Qh)
    print("NaN entries per component:", bad.sum(axis=0))
    print(periodic)
    for c in range(1):
        sel = np.nonzero(bad[:, c])[0][:3]
        for s in sel:
            cell = np.floor(X[s] * N).astype(int)
            print("comp", c, "marker", s, "cell", cell, "patch tile", cell // n, "local", cell % n)
    
for periodic in [(1, 1, 1), (1, 0, 1), (0, 1, 1), (1, 1, 0), (0, 0, 0)]:
  run(periodic)
