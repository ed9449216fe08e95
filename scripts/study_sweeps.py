"""How many gradient sweeps the gridded values need: on the C3 trace's own hits
(n^2 -> 128^2) the Chebyshev iteration's largest relative change per sweep (scipy's measure) and the
gridded Wave2 after K sweeps against a 1e-12 solve, as a fraction of the map's range.

    python scripts/study_sweeps.py [--n 3163 1001]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1001, 3163])
    ap.add_argument("--size", type=int, default=128)
    a = ap.parse_args()
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    from akbraytracing_amd.griddata import CubicGrid
    g = SystemGeometry.from_dict(json.load(open(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))))
    for n in a.n:
        out = RayWave(g, n).run()
        y, z = out["detcenter2"][1].contiguous(), out["detcenter2"][2].contiguous()
        w2 = out["wave2"].reshape(1, -1).contiguous()
        cg = CubicGrid(y, z, n, n)
        ext = cg.extent
        gx, gy = np.linspace(ext[0], ext[1], a.size), np.linspace(ext[2], ext[3], a.size)
        ref = cg.interp(w2, gx, gy, tol=1e-13).cpu().numpy()[0]
        hist = list(cg.history)
        rng = np.nanmax(ref) - np.nanmin(ref)
        gref = cg.gradients(w2, tol=1e-13)
        gabs = float(gref.abs().max())
        res = {"n": n, "range": rng, "max_abs_grad": gabs, "history_to_1e-13": hist}
        errs = {}
        for K in range(2, 31, 2):
            v = interp_k(cg, w2, gx, gy, K)
            errs[K] = float(np.nanmax(np.abs(v - ref)) / rng)
        res["value_err_frac_of_range_after_K"] = errs
        print(json.dumps(res), flush=True)


def interp_k(cg, vals, gx, gy, K):
    """interp with exactly K sweeps (maxiter = K, one batch)."""
    from akbraytracing_amd import _lib
    from akbraytracing_amd import device as D
    L = _lib.lib()
    grad = cg.gradients(vals, maxiter=K, check_every=K, adaptive=False, tol=0.0)
    gxt = torch.from_numpy(gx).to(cg.dev)
    gyt = torch.from_numpy(gy).to(cg.dev)
    mx, my = gx.size, gy.size
    owner = torch.empty(mx * my, dtype=torch.int32, device=cg.dev)
    out = torch.empty((1, my, mx), dtype=D.F64, device=cg.dev)
    _lib.check(L.akb_gd_eval_f64(*cg._tri_args(), D.ptr(gxt), mx, D.ptr(gyt), my, D.ptr(vals), D.ptr(grad), 1,
                                 D.ptr(owner), D.ptr(out), D.stream_handle()))
    return out.cpu().numpy()[0]


if __name__ == "__main__":
    main()
