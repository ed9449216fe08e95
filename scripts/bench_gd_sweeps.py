"""A/B timing of the gradient solve of the faithful chain on the C3 trace's detector-2 hits:

    python scripts/bench_gd_sweeps.py [--n 3163]

Each configuration (environment knobs of akb_gd_grad_sweeps_f64 / griddata.CubicGrid.gradients)
runs the whole solve to scipy's tolerance three times; ms = median wall time with the device
synchronised."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [
    {"AKB_GD_ROWS": "32"}, {"AKB_GD_ROWS": "48"},
    {}, {"AKB_GD_OCC": "3"}, {"AKB_GD_OCC": "2"}, {"AKB_GD_OCC": "5"}, {"AKB_GD_ROWS": "16"},
    {"AKB_GD_OCC": "2", "AKB_GD_ROWS": "16"}, {"AKB_GD_OCC": "3", "AKB_GD_ROWS": "16"},
    {"AKB_GD_OCC": "3", "AKB_GD_ROWS": "24"}, {"AKB_GD_ITER": "chebyshev-strip"},
    {"AKB_GD_RHO": "0.45"}, {"AKB_GD_RHO": "0.55"}, {"AKB_GD_RHO": "0.6"}, {"AKB_GD_ITER": "sweep"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3163)
    ap.add_argument("--cfg", default=None, help="one configuration as JSON (default: the A/B list)")
    a = ap.parse_args()
    configs = [json.loads(a.cfg)] if a.cfg else CONFIGS
    from akbraytracing_amd.griddata import CubicGrid
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    g = SystemGeometry.from_dict(json.load(open(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))))
    out = RayWave(g, a.n).run()
    y, z = out["detcenter2"][1].contiguous(), out["detcenter2"][2].contiguous()
    vals = torch.stack([out["dist_err2"], out["wave2"]])
    cg = CubicGrid(y, z, a.n, a.n)
    for cfg in configs:
        for k in ("AKB_GD_OCC", "AKB_GD_ROWS", "AKB_GD_ITER", "AKB_GD_RHO", "AKB_GD_KERNEL"):
            os.environ.pop(k, None)
        os.environ.update(cfg)
        times = []
        for _ in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            cg.gradients(vals)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t) * 1e3)
        print(json.dumps({"cfg": cfg, "ms": round(sorted(times[1:])[1], 3), "sweeps": cg.sweeps,
                          "history": [float(f"{h:.2e}") for h in cg.history]}), flush=True)


if __name__ == "__main__":
    main()
