"""Legendre basis of legendre_fit.py (:45-94), restated. TEST INFRASTRUCTURE ONLY.

aberration_legendre_component(x, y, nx, ny) = outer(P_ny(y), P_nx(x)); match_legendre
normalises it to unit nansum(Z*Z) and projects; match_legendre_multi runs degrees 0..order-1
with nx = j, ny = i - j. Pinned by tests/golden/legendre_cases.npz.
"""
import numpy as np
from numpy.polynomial import legendre as npl


def component(x, y, nx, ny):
    px = npl.legval(x, [0] * nx + [1])
    py = npl.legval(y, [0] * ny + [1])
    return np.outer(py, px)


def orders(order):
    return [(i - j, j) for i in range(order) for j in range(i + 1)]  # (ny, nx)


def fit_multi(data, order):
    xs = np.linspace(-1, 1, data.shape[0])
    ys = np.linspace(-1, 1, data.shape[1])
    fits, coefs = [], []
    for ny, nx in orders(order):
        Z = component(xs, ys, nx, ny)
        Z = Z / np.sqrt(np.nansum(Z * Z))
        c = np.nansum(Z * data)
        fits.append(c * Z)
        coefs.append(c)
    return np.array(fits), np.array(coefs)
