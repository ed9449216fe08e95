"""Debug: dump one sweep (register vs strip) on a small lattice with the diag flags."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from akbraytracing_amd.griddata import CubicGrid
from test_gpu_parity import _lattice
out = {}
for nv, nh in ((12, 10), (40, 70)):
    X, Y, F = _lattice(nv, nh, nv + nh)
    X = X * (nh / nv)
    vals = np.stack([F.ravel(), np.cos(3 * F.ravel())])
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    for it in (1, 2):
        out[f"{nv}_{it}_strip"] = cg.gradients(vals, maxiter=it, check_every=it, method="chebyshev-strip").cpu().numpy()
        out[f"{nv}_{it}_reg"] = cg.gradients(vals, maxiter=it, check_every=it, method="chebyshev").cpu().numpy()
    out[f"{nv}_diag"] = cg.diag.cpu().numpy()
    out[f"{nv}_X"], out[f"{nv}_Y"], out[f"{nv}_F"] = X, Y, vals
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "sweep_dump.npz"), **out)
