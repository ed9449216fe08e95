"""Record the reference's psf_fft_example.py computation at its own size (build container only):

    python tests/golden/make_golden_psf_example.py

psf_fft_example.py (:7-24) builds a 1024 x 1024 circular pupil (50 um pitch, radius f NA = 5 mm,
zero OPD) and calls compute_psf_fft(..., pad_factor=16): a 16384 x 16384 complex128 transform
(4 GiB; ~24 s in numpy here). The inputs are rebuilt below exactly as the example forms them;
the output is too large to commit, so psf_example.npz keeps what pins it: the shape, the peak
position, a 64 x 64 crop around the peak, the 64 x 64 grid of 256 x 256 block sums (every pixel
enters once), the central row and column every 16th sample, the total, and the image axes every
128th sample (and the last).
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402


def example_inputs():
    """psf_fft_example.py:7-24 (the commented-out defocus stays out, as in the example)"""
    wavelength_m = 13.5e-9
    focal_length_m = 0.0100
    pupil_dx_m = 50e-6
    N = 1024
    x = (np.arange(N) - N // 2) * pupil_dx_m
    X, Y = np.meshgrid(x, x, indexing='xy')
    r = np.sqrt(X**2 + Y**2)
    NA = 0.5
    R = focal_length_m * NA
    amp = (r <= R).astype(float)
    opd = np.zeros_like(amp, dtype=float)
    return opd, amp, wavelength_m, pupil_dx_m, focal_length_m


def summarize(psf, x_im, y_im):
    iy, ix = np.unravel_index(np.argmax(psf), psf.shape)
    h = 32
    B = 256
    ny, nx = psf.shape
    blocks = psf.reshape(ny // B, B, nx // B, B).sum(axis=(1, 3))
    return dict(shape=np.array(psf.shape), peak=np.array([iy, ix]),
                crop=psf[iy - h:iy + h, ix - h:ix + h].copy(), crop_origin=np.array([iy - h, ix - h]),
                blocks=blocks, row=psf[iy, ::16].copy(), col=psf[::16, ix].copy(), total=np.float64(psf.sum()),
                x_im_sub=np.r_[x_im[::128], x_im[-1]], y_im_sub=np.r_[y_im[::128], y_im[-1]])


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    import psf_fft
    opd, amp, wl, dx, f = example_inputs()
    t = time.time()
    psf, x_im, y_im = psf_fft.compute_psf_fft(opd, amp, wl, dx, f, pad_factor=16, window=None)
    el = time.time() - t
    out = summarize(psf, x_im, y_im)
    out["reference_seconds"] = np.float64(el)
    out["meta_numpy"] = np.array(np.__version__)
    np.savez_compressed(os.path.join(MG.OUT, "psf_example.npz"), **out)
    print("compute_psf_fft at", psf.shape, f"{el:.1f} s; peak", out["peak"], "total", out["total"])


if __name__ == "__main__":
    main()
