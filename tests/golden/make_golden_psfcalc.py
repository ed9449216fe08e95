"""Record the reference's post-trace path of 'ray_wave' at 65x65 (build container only; the
reference is read from /root/reference and never travels):

    python tests/golden/make_golden_psfcalc.py

Writes akb_psfcalc_65.npz with
  grid_H0, grid_V0        the interpolation grid (:3654-3657) before its mean is removed
  griddata_wave2          griddata((det2 y, z), Wave2, grid, 'cubic') (:3689)
  plane_in / plane_out    plane_correction_with_nan_and_outlier_filter(matrixWave2) in / out
                          (:3696, :9630-9693)
  psf_calc_in, grid_H, grid_V, defocus
                          the arguments of psf_calc (:3709, :1121)
  rot                     psf_calc's rotation estimate (:1122-1132), recomputed from its input
                          exactly as the reference does
  rotated                 rotate_with_nan(psf_calc_in, degrees(rot), order=3) as the opd / amp it
                          hands compute_psf_fft reveal it (amp = finite mask, opd = rotated * 1e-9)
  trim_ix / trim_iy       the indices psf_calc keeps (:1202-1223), psf_trimmed of the recorded PSF
and scipy_rotate.npz: scipy.ndimage.rotate(order=3, mode='constant', reshape=False) on random
images and angles (the third-party routine rotate_with_nan relies on; scipy pinned in meta).
Uses make_golden's stand-ins (numba, cv2, tifffile) and driver setup.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402

OUT = MG.OUT


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    import tempfile
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_psfcalc_"))
    import AKB_raytrace_20250312 as A
    import matplotlib.pyplot as plt
    import scipy
    from scipy import ndimage

    rec = {}
    orig_pc, orig_plane, orig_grid = A.psf_calc, A.plane_correction_with_nan_and_outlier_filter, A.griddata
    orig_psf = A.compute_psf_fft

    def griddata(points, values, xi, method="linear", **kw):
        r = orig_grid(points, values, xi, method=method, **kw)
        rec.setdefault("griddata", []).append((np.array(xi[0]), np.array(xi[1]), np.array(r)))
        return r

    def plane(data, *a, **k):
        r = orig_plane(data, *a, **k)
        rec.setdefault("plane", []).append((np.array(data), np.array(r)))
        return r

    def psf_calc(m, gh, gv, dw):
        rec["psf_calc"] = (np.array(m), np.array(gh), np.array(gv), float(dw))
        return orig_pc(m, gh, gv, dw)

    def psf(opd, amp, wl, dx, f, pad_factor=2, window=None, return_efield=False, pupil_dy_m=None):
        r = orig_psf(opd, amp, wl, dx, f, pad_factor=pad_factor, window=window, return_efield=return_efield,
                     pupil_dy_m=pupil_dy_m)
        rec["psf"] = (np.array(opd), np.array(amp), wl, dx, f, pad_factor, pupil_dy_m, r)
        return r

    A.griddata, A.psf_calc, A.plane_correction_with_nan_and_outlier_filter = griddata, psf_calc, plane
    A.compute_psf_fft = psf
    try:
        n = 65
        A.wave_num_H = n
        A.wave_num_V = n
        A.option_set = True
        try:
            A.plot_result_debug(MG.best_params(), "ray_wave", option_save=False)
        except Exception as e:  # the cv2 stand-in after psf_calc (:3731)
            print("stopped at:", repr(e))
    finally:
        A.griddata, A.psf_calc, A.plane_correction_with_nan_and_outlier_filter = orig_grid, orig_pc, orig_plane
        A.compute_psf_fft = orig_psf
        plt.close("all")

    m, gh, gv, dw = rec["psf_calc"]
    # psf_calc's rotation estimate (:1122-1132), computed as the reference computes it
    mins = []
    for i in range(m.shape[1]):
        v = np.where(~np.isnan(m[:, i]))[0]
        mins.append(v.min() if v.size else np.nan)
    nw = m.shape[1]
    rot = np.arctan((mins[nw // 4] - mins[nw * 3 // 4]) / (nw // 4 - nw * 3 // 4))
    opd, amp, wl, dx, f, pad, dy, (img, x_im, y_im) = rec["psf"]
    rotated = np.where(amp > 0, opd * 1e9, np.nan)  # amp is the finite mask; opd was rotated * 1e-9
    ix = np.where((x_im >= -5e-7) & (x_im <= 5e-7))[0]
    iy = np.where((y_im >= -5e-7) & (y_im <= 5e-7))[0]
    gx, gy, gw = rec["griddata"][-1]
    pin, pout = rec["plane"][0]
    np.savez_compressed(
        os.path.join(OUT, "akb_psfcalc_65.npz"),
        grid_H0=gx, grid_V0=gy, griddata_wave2=gw, plane_in=pin, plane_out=pout,
        psf_calc_in=m, grid_H=gh, grid_V=gv, defocus=np.float64(dw), rot=np.float64(rot),
        rotated=rotated, rotated_opd=opd, rotated_amp=amp, wavelength=np.float64(wl), pupil_dx=np.float64(dx),
        pupil_dy=np.float64(dy), pad=np.int64(pad), trim_ix=ix, trim_iy=iy,
        psf_trimmed=img[np.ix_(iy, ix)], x_im=x_im, y_im=y_im,
        meta=np.array(f"numpy {np.__version__} scipy {scipy.__version__}"),
    )

    rng = np.random.default_rng(7)
    cases = {}
    for k, (shape, ang) in enumerate((((23, 19), 7.3), ((66, 66), -1.2), ((40, 64), 33.0), ((17, 17), 0.4))):
        img = rng.standard_normal(shape)
        mask = (rng.random(shape) > 0.1).astype(float)
        cases[f"k{k}_in"] = img
        cases[f"k{k}_mask"] = mask
        cases[f"k{k}_angle"] = np.float64(ang)
        cases[f"k{k}_out"] = ndimage.rotate(img, ang, reshape=False, order=3, mode="constant", cval=0.0)
        cases[f"k{k}_mask_out"] = ndimage.rotate(mask, ang, reshape=False, order=3, mode="constant", cval=0.0)
    cases["meta"] = np.array(f"scipy {scipy.__version__}")
    np.savez_compressed(os.path.join(OUT, "scipy_rotate.npz"), **cases)
    print("rot", rot, "psf_calc in", m.shape, "nan", np.isnan(m).sum())


if __name__ == "__main__":
    main()
