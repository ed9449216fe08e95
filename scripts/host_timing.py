"""Time the host-side pieces of RayWave.run on this machine (resample path, ctypes launches)."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from akbraytracing_amd.wavefront import RayWave, SystemGeometry, resample_axis

g = SystemGeometry.load("tests/golden/akb_geometry.json")
n = 3163
rh, rv = g.angle_h.table(n), g.angle_v.table(n)
sh = np.tan(rh) * 1.01
sv = np.tan(rv) * 0.99
th = np.empty(2 * n)


def T(f, k=200):
    f()
    t = time.perf_counter()
    for _ in range(k):
        f()
    return (time.perf_counter() - t) / k * 1e6


def resample_all():
    np.tan(resample_axis(np.arctan(sh), rh), out=th[:n])
    np.tan(resample_axis(np.arctan(sv), rv), out=th[n:])


print("resample+arctan+tan us", T(resample_all))
print("arctan us", T(lambda: np.arctan(sh)))
print("resample_axis us", T(lambda: resample_axis(sh, rh)))
print("tan us", T(lambda: np.tan(rh)))
if torch.cuda.is_available():
    rw = RayWave(g, n)
    for _ in range(3):
        rw.run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        rw.run()
    torch.cuda.synchronize()
    print("run ms", (time.perf_counter() - t) / 10 * 1e3)
    import cProfile, pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        rw.run()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
