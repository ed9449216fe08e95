"""Record KB_debug's 'ray_wave' mode up to psf_calc (build container only; the reference is read
from /root/reference and never travels):

    python tests/golden/make_golden_kb_raywave.py

KB_debug(params, 1, 1, 'ray_wave') (AKB_raytrace_20250312.py:11725-11805) traces the KB pair once
on a wave_num_H x wave_num_V grid (no equal-angle resample: :11001 excludes the mode), tilts by the
np.mean exit angles (:11703-11717), forms DistError2 / Sph / Wave2 with np.mean (:11740-11779),
grids Wave2 with griddata(cubic) (:11783), plane-corrects it and calls psf_calc; cv2's stand-in
stops it at extract_affine_square_region. Recorded per case c (params of kb_build.npz's cases 0
and 1, n = 65 and 33, option_AKB False, option_HighNA True, EUV):

  c{c}_params, c{c}_n
  c{c}_det2          the griddata points' (y, z) rows (2, n^2): detcenter2 on the tilted rays
  c{c}_wave2         the griddata values (n^2,): Wave2
  c{c}_grid_H0 / _V0 the interpolation grid (:11756-11759)
  c{c}_plane_out     plane_correction_with_nan_and_outlier_filter's output (psf_calc's input)
  c{c}_defocus_wave  psf_calc's defocusWave
Uses make_golden's stand-ins (numba, cv2, tifffile).
"""
import contextlib
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402


def main():
    MG._stub_modules()
    sys.modules["tifffile"].imwrite = lambda *a, **kw: None  # KB_debug writes a .tiff (:11787)
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_kbrw_"))
    import AKB_raytrace_20250312 as A
    kb = np.load(os.path.join(MG.OUT, "kb_build.npz"))
    out = {}
    orig_pc, orig_plane, orig_grid = A.psf_calc, A.plane_correction_with_nan_and_outlier_filter, A.griddata
    A.option_AKB = False
    for c, (k, n) in enumerate(((0, 65), (1, 65), (1, 33))):
        rec = {}

        def griddata(points, values, xi, method="linear", **kw):
            r = orig_grid(points, values, xi, method=method, **kw)
            rec["griddata"] = (np.array(points[0]), np.array(points[1]), np.array(values), np.array(xi[0]),
                               np.array(xi[1]))
            return r

        def plane(data, *a, **kw):
            r = orig_plane(data, *a, **kw)
            rec["plane_out"] = np.array(r)
            return r

        def psf_calc(m, gh, gv, dw):
            rec["dw"] = float(dw)
            raise StopIteration  # the PSF path is pinned by akb_psfcalc_65.npz

        A.griddata, A.psf_calc, A.plane_correction_with_nan_and_outlier_filter = griddata, psf_calc, plane
        A.wave_num_H = A.wave_num_V = n
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                A.KB_debug(kb[f"k{k}_params"].copy(), 1, 1, "ray_wave", option_legendre=True, option_save=False)
        except StopIteration:
            pass
        finally:
            A.griddata, A.psf_calc, A.plane_correction_with_nan_and_outlier_filter = orig_grid, orig_pc, orig_plane
        y, z, w, gh, gv = rec["griddata"]
        out[f"c{c}_params"] = kb[f"k{k}_params"]
        out[f"c{c}_n"] = np.int64(n)
        out[f"c{c}_det2"] = np.stack([y, z])
        out[f"c{c}_wave2"] = w
        out[f"c{c}_grid_H0"] = gh
        out[f"c{c}_grid_V0"] = gv
        out[f"c{c}_plane_out"] = rec["plane_out"]
        out[f"c{c}_defocus_wave"] = np.float64(rec["dw"])
        print("case", c, "n", n, "PV", np.nanmax(rec["plane_out"]) - np.nanmin(rec["plane_out"]), "dw", rec["dw"])
    A.option_AKB = True
    out["meta_numpy"] = np.array(np.__version__)
    import scipy
    out["meta_scipy"] = np.array(scipy.__version__)
    np.savez_compressed(os.path.join(MG.OUT, "kb_raywave.npz"), **out)
    print("wrote", os.path.join(MG.OUT, "kb_raywave.npz"))


if __name__ == "__main__":
    main()
