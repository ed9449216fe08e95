"""Stage times of the faithful PSF chain (bench.py's faithful_psf_chain_ms) on the C3 trace's own
detector-2 hits (3163^2 rays -> a 128^2 pupil grid):

    python scripts/bench_faithful.py [--n 3163] [--size 128] [--reps 3]

Each stage runs with the device synchronised before and after (host steps included), ms.
"""
import argparse
import cProfile
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3163)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cprofile", action="store_true")
    a = ap.parse_args()
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    from akbraytracing_amd import pupilmap as PM
    from akbraytracing_amd.griddata import CubicGrid
    from akbraytracing_amd.psfcalc import psf_calc
    g = SystemGeometry.from_dict(json.load(open(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))))
    rw = RayWave(g, a.n)
    out = rw.run()
    det2, e2, w2 = out["detcenter2"].clone(), out["dist_err2"].clone(), out["wave2"].clone()
    n = a.n
    y, z = det2[1].contiguous(), det2[2].contiguous()

    def timed(f):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = f()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - t) * 1e3

    res = []
    for rep in range(a.reps + 1):
        row = {}
        ext = torch.stack([y.min(), y.max(), z.min(), z.max()]).cpu().numpy()
        gx = np.linspace(ext[0], ext[1], a.size)
        gy = np.linspace(ext[2], ext[3], a.size)
        cg, row["triangulate"] = timed(lambda: CubicGrid(y, z, n, n))
        vals = torch.stack([e2, w2])
        gr, row["gradients"] = timed(lambda: cg.gradients(vals))
        row["sweeps"] = cg.sweeps
        _, row["interp_incl_gradients"] = timed(lambda: cg.interp(vals, gx, gy))
        m, row["wave_maps"] = timed(lambda: PM.wave_maps(det2, e2, w2, n, n, grid_num_H=a.size, grid_num_V=a.size))
        _, row["psf_calc"] = timed(lambda: psf_calc(m["matrixWave2_Corrected"], m["grid_H"], m["grid_V"], 1e-2))
        if rep:
            res.append(row)
            print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in row.items()}), flush=True)
    if a.cprofile:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(3):
            m = PM.wave_maps(det2, e2, w2, n, n, grid_num_H=a.size, grid_num_V=a.size)
            psf_calc(m["matrixWave2_Corrected"], m["grid_H"], m["grid_V"], 1e-2)
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
