"""numpy restatement of the Wavecalc Huygens sum. TEST INFRASTRUCTURE ONLY.

forward_propagation_numpy_batch (Wavecalc_raytrace_fromData_CPU0402.py:87-124) scales the
source field by dS (:102) and, per target, sums (1/r) exp(i (-k r)) u_j over all sources
(compute_u_parallel :71-85). Pinned by tests/golden/huygens_cases.npz.
"""
import numpy as np


def propagate(tx, ty, tz, sx, sy, sz, u, k, ds, chunk=64):
    w = np.asarray(u, dtype=np.complex128) * np.asarray(ds, dtype=np.float64)
    out = np.empty(len(tx), dtype=np.complex128)
    for i0 in range(0, len(tx), chunk):
        sl = slice(i0, i0 + chunk)
        r = np.sqrt((tx[sl, None] - sx[None, :]) ** 2 + (ty[sl, None] - sy[None, :]) ** 2
                    + (tz[sl, None] - sz[None, :]) ** 2)
        out[sl] = np.sum((1.0 / r) * np.exp(1j * (-k * r)) * w[None, :], axis=1)
    return out
