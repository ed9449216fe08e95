"""Legendre figure-error model on the ray grid (BASELINE config 5).

The basis is legendre_fit's (legendre_fit.py:45-94): aberration_legendre_component(x, y, nx, ny)
= outer(P_ny(y), P_nx(x)) on x, y = linspace(-1, 1), normalised to unit norm as match_legendre
does (:70), degrees nx + ny < order in match_legendre_multi's order (ny = i - j, nx = j). Config 5
 perturbs each ray's optical path by sum_k c_k Z_k(ih, iv) with
c = 0.01 lambda default_rng(0).standard_normal(15) — a build-defined model (the reference has no
such run), so its parity is against the numpy model in oracle/legendre.py, not the reference.

The chain kernel takes it as two small tables per system: with Z_k = Py_k Px_k^T / (|Py_k| |Px_k|)
the sum is sum_ny Pv[ny][iv] * H[ny][ih], Pv = P_ny(y)/|P_ny(y)|, H = sum_nx c[ny][nx] P_nx(x)/|P_nx(x)|,
so a ray adds `order` products (akb_chain_desc.pert_h / pert_v).
"""
import numpy as np
from numpy.polynomial import legendre as npl
import torch

from . import device as D


def orders(order=5):
    """(ny, nx) pairs in match_legendre_multi's order."""
    return [(i - j, j) for i in range(order) for j in range(i + 1)]


def component(x, y, nx, ny):
    """aberration_legendre_component: outer(P_ny(y), P_nx(x))."""
    return np.outer(npl.legval(y, [0] * ny + [1]), npl.legval(x, [0] * nx + [1]))


def config5_coefficients(wavelength_m=13.5e-9, order=5, seed=0):
    return 0.01 * wavelength_m * np.random.default_rng(seed).standard_normal(len(orders(order)))


class LegendrePerturbation:
    """sum_k coeffs[k] * unit-norm Z_k over an n_h x n_v ray grid, as the two device tables the
    chain kernel reads."""

    def __init__(self, coeffs, order=5):
        self.order = int(order)
        self.coeffs = np.asarray(coeffs, dtype=np.float64)
        if self.coeffs.shape != (len(orders(self.order)),):
            raise ValueError(f"{len(orders(self.order))} coefficients expected for order {self.order}")
        if self.order > 8:
            raise ValueError("order <= 8 (the kernel sums at most 8 row terms)")

    def tables(self, n_h, n_v):
        x = np.linspace(-1, 1, n_h)
        y = np.linspace(-1, 1, n_v)
        px = [npl.legval(x, [0] * k + [1]) for k in range(self.order)]
        py = [npl.legval(y, [0] * k + [1]) for k in range(self.order)]
        pxn = [p / np.linalg.norm(p) for p in px]
        pv = np.stack([p / np.linalg.norm(p) for p in py])
        ph = np.zeros((self.order, n_h))
        for c, (ny, nx) in zip(self.coeffs, orders(self.order)):
            ph[ny] += c * pxn[nx]
        return ph, pv

    def device_tables(self, n_h, n_v, dev=None):
        ph, pv = self.tables(n_h, n_v)
        dev = dev or D.device()
        return torch.from_numpy(ph).to(dev), torch.from_numpy(pv).to(dev)

    def grid(self, n_h, n_v):
        """The perturbation itself on the grid (n_v, n_h), for checks."""
        ph, pv = self.tables(n_h, n_v)
        return pv.T @ ph
