"""Huygens-Fresnel stage timing (row a11): pairs/s of akb_huygens_f64 on BASELINE config 2's
M2 -> image stage shape: the 1e7 mirror points of a traced grid as sources
(positions from the AKB trace's last mirror, unit field, dS = 1) onto a 65 x 65 image grid
around the focus; plus the source -> M1 stage (1e7 targets, one source). Prints one JSON line.

    python scripts/bench_huygens.py [--rays 1e7] [--targets 65] [--reps 3]
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rays", type=float, default=1.0e7)
    p.add_argument("--targets", type=int, default=65)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import numpy as np
    import torch
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    from akbraytracing_amd.wavecalc import propagate
    g = SystemGeometry.load(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))
    n = int(math.ceil(math.sqrt(a.rays)))
    rw = RayWave(g, n)
    out = rw.run(keep_rotated=True)
    src = out["last_hit"]
    sx, sy, sz = src[0].contiguous(), src[1].contiguous(), src[2].contiguous()
    m = sx.shape[0]
    u = torch.ones(m, dtype=torch.complex128, device=sx.device)
    # image grid: a 2 um square around the mean detector-2 hit
    c = out["detcenter2"].mean(dim=1).cpu().numpy()
    t = np.linspace(-1e-6, 1e-6, a.targets)
    ty, tz = np.meshgrid(c[1] + t, c[2] + t)
    tx = np.full(ty.size, c[0])
    dev = sx.device
    T = [torch.from_numpy(np.ascontiguousarray(v.ravel())).to(dev) for v in (tx, ty, tz)]
    k = 2 * np.pi / 13.5e-9
    res = {}
    for name, (targ, srcs, uu) in {
        "m2_to_image": (T, (sx, sy, sz), u),
        "source_to_m1": ((sx, sy, sz), tuple(torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(3)),
                         torch.ones(1, dtype=torch.complex128, device=dev)),
    }.items():
        propagate(*targ, *srcs, uu, k)  # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            propagate(*targ, *srcs, uu, k)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        pairs = targ[0].shape[0] * srcs[0].shape[0]
        res[name] = {"targets": int(targ[0].shape[0]), "sources": int(srcs[0].shape[0]), "ms": ms,
                     "pairs_per_s": pairs / (ms * 1e-3)}
    print(json.dumps({"metric": "Huygens-Fresnel source-target pairs/s", "unit": "pairs/s", "dtype": "f64",
                      "stages": res}), flush=True)


if __name__ == "__main__":
    main()
