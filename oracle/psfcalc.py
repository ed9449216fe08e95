"""psf_calc of AKB_raytrace_20250312.py (:1121-1278), restated. TEST INFRASTRUCTURE ONLY.

Steps: the rotation estimate from the first valid row of columns n/4 and 3n/4 (:1122-1132);
rotate_with_nan (:1138-1167) = scipy.ndimage.rotate(order 3, mode 'constant', reshape=False) of
the NaN-filled map and of its mask, divided, NaN where the rotated mask < 0.5; the wavelength of
option_energy (:1161-1166); opd = map * 1e-9 with NaN -> 0 and amp = finite mask (:1182-1188);
compute_psf_fft(pad 16, pupil_dy_m) (:1200); the +-5e-7 m trim (:1202-1223).

scipy.ndimage.rotate (scipy 1.15, third party) is restated from its published algorithm: the
cubic B-spline prefilter along each axis (pole sqrt(3) - 2, gain 6, mirror-symmetric causal /
anti-causal initialisation, which scipy also uses for mode 'constant'), then at each output pixel
o the input point M o + offset, M = [[cosdg, sindg], [-sindg, cosdg]], offset = c - M c with c the
array centre; a point outside [0, n - 1] on either axis gives cval, any other point the 4 x 4
cubic B-spline sum over mirror-extended coefficients. Pinned by tests/golden/scipy_rotate.npz
(scipy's own output) and by akb_psfcalc_65.npz (the reference's psf_calc on its 65x65 run).
"""
import numpy as np
from scipy.special import cosdg, sindg

from . import psf as OP

_Z = np.sqrt(3.0) - 2.0


def spline_filter1d(x):
    """scipy.ndimage.spline_filter1d(x, order=3, mode='mirror' / 'constant') of a 1-D array."""
    z = _Z
    c = np.array(x, dtype=np.float64) * ((1.0 - z) * (1.0 - 1.0 / z))
    n = c.shape[0]
    if n == 1:
        return c
    zn1 = z ** (n - 1)
    c0 = c[0] + zn1 * c[n - 1]
    zi = z
    for i in range(1, n - 1):
        c0 += zi * (c[i] + zn1 * c[n - 1 - i])
        zi *= z
    c[0] = c0 / (1.0 - zn1 * zn1)
    for i in range(1, n):
        c[i] += z * c[i - 1]
    c[n - 1] = (z * c[n - 2] + c[n - 1]) * z / (z * z - 1.0)
    for i in range(n - 2, -1, -1):
        c[i] = z * (c[i + 1] - c[i])
    return c


def spline_filter(img):
    out = np.apply_along_axis(spline_filter1d, 0, np.asarray(img, dtype=np.float64))
    return np.apply_along_axis(spline_filter1d, 1, out)


def _mirror(i, n):
    if n == 1:
        return np.zeros_like(i)
    p = 2 * n - 2
    i = np.abs(i) % p
    return np.where(i >= n, p - i, i)


def _weights(t):
    return np.stack([(1 - t) ** 3 / 6, (4 - 6 * t * t + 3 * t ** 3) / 6,
                     (1 + 3 * t + 3 * t * t - 3 * t ** 3) / 6, t ** 3 / 6])


def rotation(shape, angle_deg):
    """(M, offset) of scipy.ndimage.rotate(reshape=False) for a 2-D array."""
    c, s = cosdg(angle_deg), sindg(angle_deg)
    M = np.array([[c, s], [-s, c]])
    centre = (np.asarray(shape, dtype=np.float64) - 1) / 2
    return M, centre - M @ centre


def rotate(img, angle_deg, cval=0.0):
    """scipy.ndimage.rotate(img, angle_deg, reshape=False, order=3, mode='constant', cval)."""
    img = np.asarray(img, dtype=np.float64)
    coef = spline_filter(img)
    ny, nx = img.shape
    M, off = rotation(img.shape, angle_deg)
    oi, oj = np.meshgrid(np.arange(ny), np.arange(nx), indexing="ij")
    y = M[0, 0] * oi + M[0, 1] * oj + off[0]
    x = M[1, 0] * oi + M[1, 1] * oj + off[1]
    inside = (y >= 0) & (y <= ny - 1) & (x >= 0) & (x <= nx - 1)
    fy, fx = np.floor(y), np.floor(x)
    wy, wx = _weights(y - fy), _weights(x - fx)
    out = np.zeros(img.shape)
    for a in range(4):
        iy = _mirror(fy.astype(np.int64) - 1 + a, ny)
        for b in range(4):
            ix = _mirror(fx.astype(np.int64) - 1 + b, nx)
            out += wy[a] * wx[b] * coef[iy, ix]
    return np.where(inside, out, cval)


def rotate_with_nan(data, angle_deg):
    """rotate_with_nan(data, angle, order=3) of psf_calc (:1138-1156)."""
    mask = (~np.isnan(data)).astype(float)
    filled = np.nan_to_num(data, nan=0.0)
    rf = rotate(filled, angle_deg)
    rm = rotate(mask, angle_deg)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = rf / np.maximum(rm, 1e-12)
    out[rm < 0.5] = np.nan
    return out


def rotation_estimate(m):
    """psf_calc's rot (:1122-1132)."""
    mins = []
    for i in range(m.shape[1]):
        v = np.where(~np.isnan(m[:, i]))[0]
        mins.append(v.min() if v.size else np.nan)
    nw = m.shape[1]
    return np.arctan((mins[nw // 4] - mins[nw * 3 // 4]) / (nw // 4 - nw * 3 // 4))


WAVELENGTH = {"EUV": 13.5e-9, "hardXray": 1.35e-10, "softXray": 1.35e-9}


def trim_half_width(option_energy, option_AKB=True):
    return 5e-8 if (option_energy == "hardXray" and option_AKB) else 5e-7


def psf_calc(m, grid_H, grid_V, defocus, option_energy="EUV", option_AKB=True):
    rot = rotation_estimate(m)
    rotated = rotate_with_nan(m, np.degrees(rot))
    wl = WAVELENGTH[option_energy]
    dx = np.abs(grid_H[0, 1] - grid_H[0, 0])
    dy = np.abs(grid_V[1, 0] - grid_V[0, 0])
    amp = np.ones_like(rotated)
    nan = np.isnan(rotated)
    amp[nan] = 0.0
    opd = rotated * 1e-9
    opd[nan] = 0.0
    psf, x_im, y_im = OP.psf(opd, amp, wl, dx, defocus, 16, dy=dy)
    h = trim_half_width(option_energy, option_AKB)
    ix = np.where((x_im >= -h) & (x_im <= h))[0]
    iy = np.where((y_im >= -h) & (y_im <= h))[0]
    return dict(rot=rot, rotated=rotated, psf=psf, x_im=x_im, y_im=y_im, psf_trimmed=psf[np.ix_(iy, ix)],
                x_trimmed=x_im[ix], y_trimmed=y_im[iy])
