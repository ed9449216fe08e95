"""Row f1 at scale: the driver's gridding step (griddata cubic x2 + nanmean + plane corrections)
on an n x n ray grid's detector hits, device vs scipy.

    python scripts/bench_griddata.py [--n 3163] [--scipy-n 401]

Prints one JSON line per measurement: stage times (HIP events on the launch stream), Jacobi
sweeps, and the agreement with scipy.interpolate.griddata on a smaller grid (scipy at 1e7 points
takes minutes; --scipy-n sets the size it is timed and compared at).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def lattice(n, seed=0):
    u, v = np.meshgrid(np.linspace(-1, 1, n), np.linspace(-1, 1, n))
    X = u * 1e-4 + 3e-6 * v ** 2 - 2e-6 * u * v + 1e-6 * v ** 3
    Y = v * 1.3e-4 + 4e-6 * u ** 2 + 1e-6 * u ** 3
    rng = np.random.default_rng(seed)
    F = 0.3 * u ** 2 - 0.2 * u * v + 0.1 * np.sin(3 * v) + 1e-3 * rng.standard_normal(u.shape)
    return X, Y, F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3163)
    ap.add_argument("--scipy-n", type=int, default=401)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from akbraytracing_amd import device as D
    from akbraytracing_amd.griddata import CubicGrid
    from akbraytracing_amd import pupilmap as PM

    n = a.n
    X, Y, F = lattice(n)
    dev = D.device()
    x = torch.from_numpy(X.ravel()).to(dev)
    y = torch.from_numpy(Y.ravel()).to(dev)
    f = torch.from_numpy(np.stack([F.ravel(), 2 * F.ravel()])).to(dev)
    gx = np.linspace(X.min(), X.max(), n)
    gy = np.linspace(Y.min(), Y.max(), n)
    det = torch.stack([torch.zeros_like(x), x, y])
    for rep in range(a.reps + 1):
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        ev[0].record()
        cg = CubicGrid(x, y, n, n)
        ev[1].record()
        g = cg.gradients(f)
        ev[2].record()
        out = cg.interp(f, gx, gy)  # includes its own gradient solve
        ev[3].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if rep:
            print(json.dumps({"what": "griddata_device", "n_points": n * n, "value_sets": 2,
                              "triangulate_ms": ev[0].elapsed_time(ev[1]), "gradients_ms": ev[1].elapsed_time(ev[2]),
                              "interp_ms": ev[2].elapsed_time(ev[3]), "sweeps": cg.sweeps, "npockets": cg.npock,
                              "wall_s": wall}), flush=True)
    for rep in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = PM.wave_maps(det, f[0], f[1], n, n)
        torch.cuda.synchronize()
        if rep:
            print(json.dumps({"what": "wave_maps_device", "n_points": n * n, "wall_ms": 1e3 * (time.perf_counter() - t0),
                              "sweeps": r["sweeps"]}), flush=True)
    del out, g, r
    from scipy.interpolate import griddata as sp_griddata
    m = a.scipy_n
    X, Y, F = lattice(m)
    gx = np.linspace(X.min(), X.max(), m)
    gy = np.linspace(Y.min(), Y.max(), m)
    GH, GV = np.meshgrid(gx, gy)
    t0 = time.perf_counter()
    want = sp_griddata((X.ravel(), Y.ravel()), F.ravel(), (GH, GV), method="cubic")
    t_sp = time.perf_counter() - t0
    cg = CubicGrid(X.ravel(), Y.ravel(), m, m)
    got = cg.interp(F.ravel(), gx, gy)[0].cpu().numpy()
    same_nan = bool(np.array_equal(np.isnan(got), np.isnan(want)))
    d = np.abs(got - want)
    rng = float(np.nanmax(want) - np.nanmin(want))
    print(json.dumps({"what": "scipy_compare", "n_points": m * m, "scipy_s": t_sp, "same_nan_mask": same_nan,
                      "max_abs_diff": float(np.nanmax(d)), "rms_diff": float(np.sqrt(np.nanmean(d ** 2))),
                      "range": rng}), flush=True)


if __name__ == "__main__":
    main()
