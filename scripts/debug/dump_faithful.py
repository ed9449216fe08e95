"""Debug: device wave_maps at n x n onto 128^2 with each gradient iteration; saves the maps."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from akbraytracing_amd.wavefront import RayWave, SystemGeometry
from akbraytracing_amd import pupilmap as PM
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1001
g = SystemGeometry.from_dict(json.load(open(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))))
out = RayWave(g, n).run(full=True)
res = {}
for meth in ("chebyshev", "chebyshev-strip", "sweep"):
    os.environ["AKB_GD_ITER"] = meth
    r = PM.wave_maps(out["detcenter2"], out["dist_err2"], out["wave2"], n, n, grid_num_H=128, grid_num_V=128)
    for k in ("matrixWave2", "matrixDistError2", "matrixWave2_Corrected", "matrixDistError2_Corrected"):
        res[f"{meth}_{k}"] = r[k].cpu().numpy()
    res[f"{meth}_sweeps"] = np.array(r["sweeps"])
    print(meth, r["sweeps"], flush=True)
res["det2"] = out["detcenter2"].cpu().numpy()
res["wave2"] = out["wave2"].cpu().numpy()
res["dist_err2"] = out["dist_err2"].cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"dump_faithful_{n}.npz"), **res)
