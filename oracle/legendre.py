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


def config5_coefficients(wavelength_m=13.5e-9, order=5, seed=0):
    """BASELINE config 5's figure-error coefficients: c = 0.01 lambda N(0, 1)
    from numpy's default_rng(seed), one per (ny, nx) of orders(order)."""
    return 0.01 * wavelength_m * np.random.default_rng(seed).standard_normal(len(orders(order)))


def perturbation(n_h, n_v, coeffs, order=5):
    """sum_k c_k Z_k on the n_v x n_h ray grid, Z_k the unit-norm component of match_legendre
    (x = linspace(-1, 1) over ih, y over iv): the per-ray OPL perturbation of config 5."""
    xs = np.linspace(-1, 1, n_h)
    ys = np.linspace(-1, 1, n_v)
    out = np.zeros((n_v, n_h))
    for c, (ny, nx) in zip(coeffs, orders(order)):
        Z = component(xs, ys, nx, ny)
        out += c * (Z / np.sqrt(np.nansum(Z * Z)))
    return out
