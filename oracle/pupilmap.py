"""plane_correction_with_nan_and_outlier_filter (AKB_raytrace_20250312.py:9630-9693), restated.
TEST INFRASTRUCTURE ONLY: the checker for akbraytracing_amd.pupilmap, never the product path.

The reference fits the quadratic a x + b y + c + d x^2 + e y^2 and then the plane a x + b y + c
with scipy's curve_fit; both models are linear in their parameters, so the fits are linear least
squares, restated here with np.linalg.lstsq on the same index coordinates. Pinned by
tests/golden/akb_psfcalc_65.npz (plane_in -> plane_out, the reference's own output): agreement
~4e-14 nm on a 0.23 nm range (curve_fit stops at its own tolerance; not bit-exact).
"""
import numpy as np


def plane_correction_with_nan_and_outlier_filter(data, sigma_threshold=3):
    x, y = np.meshgrid(np.arange(data.shape[1]), np.arange(data.shape[0]))
    mask = ~np.isnan(data)
    xf, yf, zf = x[mask].astype(np.float64), y[mask].astype(np.float64), data[mask]
    A1 = np.stack([xf, yf, np.ones_like(xf), xf ** 2, yf ** 2], axis=1)
    p1 = np.linalg.lstsq(A1, zf, rcond=None)[0]
    res = zf - A1 @ p1
    keep = np.abs(res) < sigma_threshold * np.std(res)
    A2 = np.stack([xf[keep], yf[keep], np.ones(int(keep.sum()))], axis=1)
    p2 = np.linalg.lstsq(A2, zf[keep], rcond=None)[0]
    out = data - (p2[0] * x + p2[1] * y + p2[2])
    out[~mask] = np.nan
    return out
