"""Wall time of plot_result_debug(params, 'ray_wave', option_legendre=True) on the device
(akbraytracing_amd/driver.py: build, trace, tilt, OPD, griddata, plane correction, psf_calc,
rectification, Legendre fit, files) for the best-alignment params at several grid sizes:

    python scripts/bench_driver.py [--sizes 65 1001 3163] [--reps 3] [--out gpurun_out/driver.json]

The reference's own run of that mode at 65^2 took 1.23 s up to its cv2 step on one core of the
survey container; its 'wave' trace alone took 36.3 s at 3163^2.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def best_params():
    p = np.zeros(26)  # AKB_raytrace_20250312.py:14586-14592
    p[0], p[1], p[8], p[9], p[13] = -5.73452570e-03, -2.87624337e-03, 1.05000000e-02, -3.59399021e-05, 2.39536993e-06
    p[20], p[21], p[25] = 1.05000000e-02, -3.59399021e-05, 2.39536993e-06
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[65, 1001, 3163])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from akbraytracing_amd.driver import plot_result_ray_wave
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for n in a.sizes:
            times = []
            for rep in range(a.reps + 1):
                torch.cuda.synchronize()
                t = time.perf_counter()
                plot_result_ray_wave(best_params(), n, directory=tmp, workdir=tmp, verbose=False)
                torch.cuda.synchronize()
                if rep:
                    times.append((time.perf_counter() - t) * 1e3)
            res[str(n)] = dict(ms_median=float(np.median(times)), ms=times, rays=n * n)
            print(json.dumps({n: res[str(n)]}), flush=True)
    res["reference_65_s"] = 1.23
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
