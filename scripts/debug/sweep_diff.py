"""Debug: register-kernel sweeps vs the strip kernel's Chebyshev sweeps on test lattices."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from akbraytracing_amd.griddata import CubicGrid
from test_gpu_parity import _lattice
for nv, nh, nvals in ((40, 70, 1), (40, 70, 2), (97, 113, 2), (300, 280, 1), (300, 280, 2), (97, 113, 1), (70, 530, 2), (33, 257, 2)):
    X, Y, F = _lattice(nv, nh, nv + nh)
    X = X * (nh / nv)
    vals = np.stack([F.ravel(), np.cos(3 * F.ravel())])[:nvals]
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    for it in (1, 2, 3, 5):
        a = cg.gradients(vals, maxiter=it, check_every=it, method="chebyshev-strip").cpu().numpy()
        b = cg.gradients(vals, maxiter=it, check_every=it, method="chebyshev").cpu().numpy()

        bad = np.argwhere(np.any(a != b, axis=-1))
        msg = f"{nv}x{nh} nv={nvals} it={it}: {len(bad)} differ"
        if len(bad):
            v, i = bad[0]
            msg += f"; first set {v} vertex {i} = (iv {i // nh}, ih {i % nh}) strip {a[v, i]} reg {b[v, i]}"
            rows = sorted(set((bad[:, 1] // nh).tolist()))
            cols = sorted(set((bad[:, 1] % nh).tolist()))
            msg += f" rows {rows[:10]}.. cols {cols[:10]}.."
        print(msg, flush=True)
