"""numpy restatement of psf_fft.compute_psf_fft (psf_fft.py:29-125). TEST INFRASTRUCTURE ONLY.

Steps, in the reference's order: NaN/inf -> 0 in opd and amp; U = A exp(i 2pi/lambda opd);
optional separable Hann (unit peak); pad odd sides by one; centred zero-pad by pad_factor;
fftshift(fft2(ifftshift(U))) * dx dy; I = |U|^2 / max. Pinned by tests/golden/psf_cases.npz.
"""
import numpy as np


def psf(opd_m, amp, wavelength_m, dx, focal_length_m, pad_factor=2, window=None, return_efield=False, dy=None):
    A = np.nan_to_num(np.asarray(amp, dtype=float), nan=0.0, posinf=0.0, neginf=0.0)
    o = np.nan_to_num(np.asarray(opd_m, dtype=float), nan=0.0, posinf=0.0, neginf=0.0)
    field = A * np.exp(1j * ((2.0 * np.pi / wavelength_m) * o))
    ny, nx = field.shape
    if window is not None:
        wy = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(ny) / ny)
        wx = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(nx) / nx)
        w = np.outer(wy, wx)
        field = field * (w / w.max())
    ey, ex = ny + ny % 2, nx + nx % 2
    py, px = ey * pad_factor, ex * pad_factor
    big = np.zeros((py, px), dtype=complex)
    y0, x0 = (py - ey) // 2, (px - ex) // 2
    big[y0:y0 + ny, x0:x0 + nx] = field
    dyv = dx if dy is None else dy
    U = np.fft.fftshift(np.fft.fft2(np.fft.ifftshift(big))) * (dx * dyv)
    x_im = wavelength_m * focal_length_m * np.fft.fftshift(np.fft.fftfreq(px, d=dx))
    y_im = wavelength_m * focal_length_m * np.fft.fftshift(np.fft.fftfreq(py, d=dyv))
    I = np.abs(U) ** 2
    m = I.max()
    if m > 0:
        I = I / m
    if return_efield:
        return I, x_im, y_im, U / np.sqrt(m if m > 0 else 1.0)
    return I, x_im, y_im
