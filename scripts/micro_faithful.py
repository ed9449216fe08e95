"""The faithful chain alone (no trace kernels beside it): FaithfulPupil.run on the C3 trace's own
hits, repeated; run under rocprofv3 --kernel-trace --stats for the standalone kernel times.

    python scripts/micro_faithful.py [--n 3163] [--reps 20] [--out file.npz]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3163)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    g = SystemGeometry.from_dict(json.load(open(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))))
    out = RayWave(g, a.n).run()
    y, z, w = out["detcenter2"][1].clone(), out["detcenter2"][2].clone(), out["wave2"].clone()
    fp = FaithfulPupil(a.n, a.n, slots=2)
    ms, dev = [], []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        t = fp.begin(y, z, w)
        t.job.result()
        r = fp.finish(t, events=e)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
        dev.append(e[0].elapsed_time(e[1]))
        t.check()
    print(json.dumps({"n": a.n, "wall_ms_median": sorted(ms)[len(ms) // 2],
                      "finish_device_ms_median": sorted(dev)[len(dev) // 2]}))
    if a.out:
        np.savez(a.out, psf=r["psf"].cpu().numpy(), map=r["map"].cpu().numpy(), rotated=r["rotated"].cpu().numpy())
    fp.close()


if __name__ == "__main__":
    main()
