"""psf_calc of the 'ray_wave' driver (AKB_raytrace_20250312.py:1121-1278), device-backed.

The reference's psf_calc(matrixWave2_Corrected, grid_H, grid_V, defocusWave): estimates the
pupil's rotation from the first valid row of columns n/4 and 3n/4 (:1122-1132), rotates the map
back with rotate_with_nan(order=3) (scipy.ndimage.rotate of the NaN-filled map and of its mask,
:1138-1167), picks the wavelength of option_energy (:1161-1166), forms opd = map * 1e-9 and the
finite-mask amplitude (:1182-1188), calls compute_psf_fft(pad_factor=16, pupil_dy_m) (:1200) and
trims +-5e-7 m (+-5e-8 m for hard X-ray AKB, :1202-1223); it then plots and saves psf.npy,
psf_x.npy, psf_y.npy (:1271-1273).

Here the rotation and the PSF run on the device (akb_first_valid_rows_f64,
akb_rotate_with_nan_f64, akb_psf_f64); the two host steps are the reference's own scalar
arithmetic: np.arctan of the index slope and scipy.special.cosdg / sindg for the rotation matrix
(the functions scipy.ndimage.rotate calls). Plots are out of scope; the .npy files are written
when a directory is given.
"""
import os

import numpy as np
import torch
from scipy.special import cosdg, sindg

from . import _lib
from . import device as D
from .psf import image_axes, psf_stack

WAVELENGTH = {"EUV": 13.5e-9, "hardXray": 1.35e-10, "softXray": 1.35e-9}  # :1161-1166


def trim_half_width(option_energy, option_AKB=True):
    """Half-width of the kept PSF window in metres (:1202-1214)."""
    return 5e-8 if (option_energy == "hardXray" and option_AKB) else 5e-7


def rotation_estimate(m):
    """rot of :1122-1132 from a (ny, nx) device map: the first valid row of each column on the
    device, the slope's arctan with numpy as the reference takes it."""
    L = _lib.lib()
    ny, nx = int(m.shape[0]), int(m.shape[1])
    rows = torch.empty(nx, dtype=torch.int32, device=m.device)
    _lib.check(L.akb_first_valid_rows_f64(D.ptr(m), ny, nx, D.ptr(rows), D.stream_handle()))
    mins = [int(v) if v >= 0 else np.nan for v in rows.cpu().numpy()]  # NaN for an all-NaN column
    return np.arctan((mins[nx // 4] - mins[nx * 3 // 4]) / (nx // 4 - nx * 3 // 4))


def rotate_with_nan(m, angle_deg):
    """rotate_with_nan(m, angle, order=3) (:1138-1156) on a (ny, nx) float64 device map.
    Returns (rotated [nm, NaN outside], rotated * 1e-9) as device tensors."""
    L = _lib.lib()
    m = m.to(D.F64).contiguous()
    ny, nx = int(m.shape[0]), int(m.shape[1])
    c, s = cosdg(angle_deg), sindg(angle_deg)
    rot = np.array([[c, s], [-s, c]])
    centre = (np.array([ny, nx], dtype=np.float64) - 1) / 2
    offset = centre - rot @ centre
    out = torch.empty((ny, nx), dtype=D.F64, device=m.device)
    opd = torch.empty((ny, nx), dtype=D.F64, device=m.device)
    work = torch.empty(int(L.akb_rotate_work_bytes(ny, nx)), dtype=torch.uint8, device=m.device)
    _lib.check(L.akb_rotate_with_nan_f64(D.ptr(m), ny, nx, D.host_f64(rot.ravel()), D.host_f64(offset), D.ptr(out),
                                         D.ptr(opd), D.ptr(work), D.stream_handle()))
    return out, opd


def psf_calc(matrixWave2_Corrected, grid_H, grid_V, defocusWave, option_energy="EUV", option_AKB=True,
             directory=None):
    """The reference's psf_calc on the device. Returns a dict: rot, rotated (device, nm), psf
    (device, peak 1), x_im, y_im (numpy), psf_trimmed (device view), x_trimmed, y_trimmed; writes
    psf.npy / psf_x.npy / psf_y.npy under `directory` like :1271-1273 when one is given."""
    if option_energy not in WAVELENGTH:
        raise ValueError(f"option_energy must be one of {sorted(WAVELENGTH)}")
    m = D.to_dev(matrixWave2_Corrected) if not isinstance(matrixWave2_Corrected, torch.Tensor) else \
        matrixWave2_Corrected.to(device=D.device(), dtype=D.F64).contiguous()
    gh = np.asarray(grid_H.cpu() if isinstance(grid_H, torch.Tensor) else grid_H, dtype=np.float64)
    gv = np.asarray(grid_V.cpu() if isinstance(grid_V, torch.Tensor) else grid_V, dtype=np.float64)
    rot = rotation_estimate(m)
    rotated, opd = rotate_with_nan(m, np.degrees(rot))
    wl = WAVELENGTH[option_energy]
    dx = np.abs(gh[0, 1] - gh[0, 0])
    dy = np.abs(gv[1, 0] - gv[0, 0])
    # amp = 1 where the rotated map is defined, 0 at its NaNs; opd NaN -> 0 (:1182-1188)
    psf, _, _ = psf_stack(opd, None, [wl], dx, dy, pad_factor=16)
    ny, nx = int(m.shape[0]), int(m.shape[1])
    py, px = (ny + ny % 2) * 16, (nx + nx % 2) * 16
    x_im, y_im = image_axes(px, py, dx, dy, wl, float(defocusWave))
    h = trim_half_width(option_energy, option_AKB)
    ix = np.where((x_im >= -h) & (x_im <= h))[0]
    iy = np.where((y_im >= -h) & (y_im <= h))[0]
    img = psf[0]
    trimmed = img[int(iy[0]):int(iy[-1]) + 1, int(ix[0]):int(ix[-1]) + 1] if ix.size and iy.size else img[:0, :0]
    if directory is not None:
        os.makedirs(directory, exist_ok=True)
        np.save(os.path.join(directory, "psf.npy"), img.cpu().numpy())
        np.save(os.path.join(directory, "psf_x.npy"), x_im)
        np.save(os.path.join(directory, "psf_y.npy"), y_im)
    return dict(rot=rot, rotated=rotated, psf=img, x_im=x_im, y_im=y_im, psf_trimmed=trimmed,
                x_trimmed=x_im[ix], y_trimmed=y_im[iy])
