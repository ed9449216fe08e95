"""Fraunhofer PSF of a pupil: the reference's psf_fft module, device-backed.

compute_psf_fft / psf_to_db / ensure_even_size keep psf_fft.py's signatures, argument checks
(ValueError on a shape mismatch, a bad pad_factor, an unknown window: psf_fft.py:74-77, :92) and
return values (numpy arrays). psf_stack() is the device API: one batched 2-D transform over a
stack of wavelengths (config 5's multi-lambda PSF), inputs and outputs as device tensors.

On the device (libakb_hip.so, akb_psf_f64) the padded plane is never built: it is zero outside
the pupil block, so at pad 8 and 16 (every caller's pad) the transform runs as pruned line
transforms (k_psf_line: the pupil's columns, the peak rows, then the normalised write - DESIGN.md
§4.1); other pads of small pupils take the column-pass transform, and only the remaining shapes
build the padded, ifftshift-ed field and run rocFFT's in-place complex transform, then fftshift,
dA, |U|^2, the per-wavelength peak and the normalisation pass.
"""
import numpy as np
import torch

from . import _lib
from . import device as D

__all__ = ["compute_psf_fft", "psf_to_db", "ensure_even_size", "psf_stack", "image_axes"]


def ensure_even_size(arr):
    """psf_fft.ensure_even_size (psf_fft.py:6-18): pad odd sides by one zero at the end."""
    ny, nx = arr.shape
    py, px = ny % 2, nx % 2
    if not (py or px):
        return arr, None
    # np.pad(arr, ..., mode="constant") as psf_fft.py:15: the input dtype is kept (int, bool too)
    out = np.zeros((ny + py, nx + px), dtype=arr.dtype)
    out[:ny, :nx] = arr
    return out, (slice(0, ny), slice(0, nx))


def hann_axes(ny, nx):
    """The separable factors of psf_fft._hann2d and the peak of their outer product."""
    wx = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(nx) / nx)
    wy = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(ny) / ny)
    return wy, wx, float(np.outer(wy, wx).max())


def image_axes(px, py, dx, dy, wavelength_m, focal_length_m):
    """x_im, y_im of psf_fft.py:114-117: lambda f fftshift(fftfreq(p, d))."""
    fx = np.fft.fftshift(np.fft.fftfreq(px, d=dx))
    fy = np.fft.fftshift(np.fft.fftfreq(py, d=dy))
    return wavelength_m * focal_length_m * fx, wavelength_m * focal_length_m * fy


def _check_args(opd_shape, amp_shape, pad_factor, window):
    if tuple(opd_shape) != tuple(amp_shape):
        raise ValueError("opd_m and amp must have the same shape")
    if pad_factor < 1 or int(pad_factor) != pad_factor:
        raise ValueError("pad_factor must be a positive integer")
    if window is not None and str(window).lower() != "hann":
        raise ValueError(f"Unsupported window '{window}'. Options: 'hann' or None.")


class PsfWorkspace:
    """Reusable device buffers for repeated PSF launches of one geometry."""

    def __init__(self):
        self.work = None

    def get(self, ny, nx, pad, batch, dev):
        L = _lib.lib()
        need = int(L.akb_psf_work_bytes(ny, nx, pad, batch))
        if need < 0:
            _lib.check(-3)
        if self.work is None or self.work.numel() < need or self.work.device != dev:
            self.work = torch.empty(need, dtype=torch.uint8, device=dev)
        return self.work


_ws = PsfWorkspace()


def psf_stack(opd, amp, wavelengths, dx, dy=None, pad_factor=2, window=None, return_efield=False,
              workspace=None, stream=None, pitch=None, out=None):
    """Device API. opd, amp: (ny, nx) float64 device tensors (amp None: 1 where opd is finite,
    psf_calc's mask). wavelengths: sequence of up to 8. pitch: optional device [dx, dy] tensor
    replacing dx/dy (no host round trip). out: optional preallocated (B, py, px) psf tensor.
    Returns (psf (B, py, px), efield (B, py, px) complex128 or None, imax (B,) device tensor)."""
    L = _lib.lib()
    _check_args(opd.shape, opd.shape if amp is None else amp.shape, pad_factor, window)
    dev = opd.device
    ny, nx = int(opd.shape[0]), int(opd.shape[1])
    pad = int(pad_factor)
    lams = [float(w) for w in np.atleast_1d(wavelengths)]
    B = len(lams)
    if not 1 <= B <= 8:
        raise ValueError("1..8 wavelengths per launch")
    py, px = (ny + ny % 2) * pad, (nx + nx % 2) * pad
    psf = out if out is not None and tuple(out.shape) == (B, py, px) else torch.empty((B, py, px), dtype=D.F64,
                                                                                         device=dev)
    ef = torch.empty((B, py, px), dtype=torch.complex128, device=dev) if return_efield else None
    imax = torch.empty(B, dtype=D.F64, device=dev)
    work = (workspace or _ws).get(ny, nx, pad, B, dev)
    wy = wx = None
    wmax = 1.0
    if window is not None:
        hy, hx, wmax = hann_axes(ny, nx)
        wy, wx = D.to_dev(hy, dev), D.to_dev(hx, dev)
    dxv = 0.0 if dx is None else float(dx)
    dyv = dxv if dy is None else float(dy)
    opd_c = opd.to(D.F64).contiguous()
    amp_c = None if amp is None else amp.to(D.F64).contiguous()
    _lib.check(L.akb_psf_f64(D.ptr(opd_c), D.ptr(amp_c), ny, nx, pad, B, D.host_f64(lams), dxv, dyv,
                             D.ptr(wy), D.ptr(wx), wmax, D.ptr(psf),
                             D.ptr(torch.view_as_real(ef)) if ef is not None else None, D.ptr(imax),
                             D.ptr(pitch), D.ptr(work), D.stream_handle(stream)))
    return psf, ef, imax


def compute_psf_fft(opd_m, amp, wavelength_m, pupil_dx_m, focal_length_m, pad_factor=2, window=None,
                    return_efield=False, pupil_dy_m=None):
    """Drop-in for psf_fft.compute_psf_fft (psf_fft.py:29-125), computed on the GPU.
    Returns (psf, x_im, y_im[, efield_im]) as numpy arrays like the reference."""
    opd_np = np.asarray(opd_m)
    amp_np = np.asarray(amp)
    _check_args(opd_np.shape, amp_np.shape, pad_factor, window)
    dev = D.device()
    o = D.to_dev(opd_np.astype(float), dev)
    a = D.to_dev(amp_np.astype(float), dev)
    dy = pupil_dx_m if pupil_dy_m is None else pupil_dy_m
    psf, ef, _ = psf_stack(o, a, [wavelength_m], pupil_dx_m, dy, pad_factor=pad_factor, window=window,
                           return_efield=return_efield)
    ny, nx = opd_np.shape
    py, px = (ny + ny % 2) * int(pad_factor), (nx + nx % 2) * int(pad_factor)
    x_im, y_im = image_axes(px, py, pupil_dx_m, dy, wavelength_m, focal_length_m)
    if return_efield:
        return psf[0].cpu().numpy(), x_im, y_im, ef[0].cpu().numpy()
    return psf[0].cpu().numpy(), x_im, y_im


def psf_to_db(psf, floor_db=-60.0):
    """psf_fft.psf_to_db (psf_fft.py:127-131): 10 log10(max(psf, 10^(floor/10)))."""
    with np.errstate(divide="ignore"):
        return 10.0 * np.log10(np.maximum(psf, 10.0 ** (floor_db / 10.0)))
