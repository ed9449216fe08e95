"""Full-size fixtures beyond akb_raywave_full.npz (build container only; the reference is read from
/root/reference and never travels):

    python tests/golden/make_golden_full_extra.py psf            -> akb_psf_full.npz
    python tests/golden/make_golden_full_extra.py qhull [n ...]  -> akb_qhull_full.npz (default 1001 3163)
    python tests/golden/make_golden_full_extra.py ellipse        -> ellipse_317.npz

psf: the reference's own psf_calc (AKB_raytrace_20250312.py:1121-1278) on the reference's own
plane-corrected 128 x 128 Wave2 maps of akb_raywave_full.npz (n = 1001 and 3163), with the driver's
grid handling before the call (grid_H -= mean, grid_V -= mean, :3698-3700) and defocusWave = 1e-2
(:3613). Its compute_psf_fft call (:1200) is captured:

  n{n}_rot              the rotation estimate (:1122-1132)
  n{n}_rotated          the map after rotate_with_nan (opd / 1e-9 where amp = 1, NaN elsewhere)
  n{n}_psf_crop         the PSF (peak 1) on the trimmed window of :1202-1223 (+-5e-7 m)
  n{n}_psf_win          [iy0, iy1, ix0, ix1] of that window in the 2048^2 plane
  n{n}_psf_stats        [sum, argmax row, argmax col] of the whole plane
  n{n}_x_im, n{n}_y_im  the image axes

qhull: the reference's plot_result_debug(params, 'ray_wave') hits at n x n (the griddata points of
:3689, as make_golden_raywave_full.py records them), triangulated by scipy's Delaunay (qhull), and
for every cell whose qhull split is not the exact in-circle diagonal of akb_griddata.hip:

  n{n}_flip_cells       flat cell index iv * (n - 1) + ih
  n{n}_flip_qd          qhull's split there: 0 = p00-p11, 1 = p01-p10, -1 = neither (the cell's
                        four points are not two qhull triangles)

so a test can impose qhull's own triangulation on the device's structured one and hold the gridded
maps to the 1e-6 bar everywhere (tests/test_fullsize_gpu.py).

ellipse: BASELINE configs[0] (C1): EllipseRaytrace3D's __main__ single ellipse (:302-363) at its
num = 317 (1.0e5 rays) - calc_reflect and PlanePoints(dist_s_f, 1e-8) - recorded like ellipse_33.
"""
import contextlib
import io
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402


def _import_akb():
    MG._stub_modules()
    sys.modules["tifffile"].imwrite = lambda *a, **kw: None
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_extra_"))
    import AKB_raytrace_20250312 as A
    return A


def psf(A):
    full = np.load(os.path.join(MG.OUT, "akb_raywave_full.npz"))
    out = {}
    for n in (1001, 3163):
        m = full[f"n{n}_map_wave_c"]
        GH, GV = np.meshgrid(full[f"n{n}_gx"], full[f"n{n}_gy"])
        GH = GH - np.mean(GH)  # the driver's grid_H -= np.mean(grid_H) (:3698)
        GV = GV - np.mean(GV)
        calls = []
        orig = A.compute_psf_fft

        def capture(opd, amp, wl, dx, f, pad_factor=2, window=None, return_efield=False, pupil_dy_m=None):
            r = orig(opd, amp, wl, dx, f, pad_factor=pad_factor, window=window, return_efield=return_efield,
                     pupil_dy_m=pupil_dy_m)
            calls.append(dict(opd=np.array(opd), amp=np.array(amp), out=r))
            return r

        A.compute_psf_fft = capture
        try:
            with contextlib.redirect_stdout(io.StringIO()) as so:
                A.psf_calc(m.copy(), GH, GV, 1e-2)
        finally:
            A.compute_psf_fft = orig
        rot = float([ln for ln in so.getvalue().splitlines() if ln.startswith("rot")][0].split()[1])
        (c,) = calls
        P, x_im, y_im = c["out"]
        h = 5e-7
        ix = np.where((x_im >= -h) & (x_im <= h))[0]
        iy = np.where((y_im >= -h) & (y_im <= h))[0]
        rotated = np.where(c["amp"] > 0, c["opd"] / 1e-9, np.nan)
        am = np.unravel_index(np.argmax(P), P.shape)
        out.update({f"n{n}_rot": np.float64(rot), f"n{n}_rotated": rotated,
                    f"n{n}_psf_crop": P[iy[0]:iy[-1] + 1, ix[0]:ix[-1] + 1],
                    f"n{n}_psf_win": np.array([iy[0], iy[-1] + 1, ix[0], ix[-1] + 1]),
                    f"n{n}_psf_stats": np.array([P.sum(), am[0], am[1]], dtype=np.float64),
                    f"n{n}_x_im": x_im, f"n{n}_y_im": y_im})
        print(f"n={n}: rot {rot}, PSF {P.shape}, window {out[f'n{n}_psf_win']}", flush=True)
    np.savez_compressed(os.path.join(MG.OUT, "akb_psf_full.npz"), **out)


def qhull(A, sizes):
    from scipy.spatial import Delaunay
    path = os.path.join(MG.OUT, "akb_qhull_full.npz")
    out = dict(np.load(path)) if os.path.exists(path) else {}
    for n in sizes:
        A.wave_num_H = A.wave_num_V = n
        A.option_set = True
        grid_calls = []
        orig_grid = A.griddata

        def griddata(points, values, xi, method="linear", **kw):
            grid_calls.append((np.array(points[0]), np.array(points[1])))
            raise StopIteration

        A.griddata = griddata
        t0 = time.time()
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                A.plot_result_debug(MG.best_params(), "ray_wave", option_save=False)
        except StopIteration:
            pass
        finally:
            A.griddata = orig_grid
        y, z = grid_calls[0]
        print(f"n={n}: reference trace {time.time() - t0:.1f} s", flush=True)
        t0 = time.time()
        tri = Delaunay(np.stack([y, z], axis=1))
        print(f"n={n}: qhull {time.time() - t0:.1f} s", flush=True)
        S = np.sort(tri.simplices, axis=1).astype(np.int64)
        del tri
        a, b, c = S[:, 0], S[:, 1], S[:, 2]
        qd = np.full((n - 1) * (n - 1), -1, np.int8)

        def mark(sel, cell_vertex, d):
            iv, ih = np.divmod(cell_vertex[sel], n)
            ok = (iv < n - 1) & (ih < n - 1)
            qd[(iv * (n - 1) + ih)[ok]] = d

        # the same classification as make_golden_raywave_full.qhull_ambiguity
        mark((b == a + 1) & (c == a + n + 1), a, 0)
        mark((b == a + n) & (c == a + n + 1), a, 0)
        mark((b == a + 1) & (c == a + n), a, 1)
        mark((b == a + n - 1) & (c == a + n), a - 1, 1)
        Y, Z = y.reshape(n, n), z.reshape(n, n)
        x0, y0 = Y[:-1, :-1], Z[:-1, :-1]
        bx, by = Y[:-1, 1:] - x0, Z[:-1, 1:] - y0
        cx, cy = Y[1:, 1:] - x0, Z[1:, 1:] - y0
        dx, dy = Y[1:, :-1] - x0, Z[1:, :-1] - y0
        adx, ady, bdx, bdy, cdx, cdy = -dx, -dy, bx - dx, by - dy, cx - dx, cy - dy
        A_, B_, C_ = adx * adx + ady * ady, bdx * bdx + bdy * bdy, cdx * cdx + cdy * cdy
        det = adx * (bdy * C_ - B_ * cdy) - ady * (bdx * C_ - B_ * cdx) + A_ * (bdx * cdy - bdy * cdx)
        o = bx * cy - by * cx
        exact = (np.where(o > 0, det, -det) > 0).astype(np.int8).ravel()
        cells = np.nonzero(qd != exact)[0]
        out[f"n{n}_flip_cells"] = cells.astype(np.int64)
        out[f"n{n}_flip_qd"] = qd[cells]
        print(f"n={n}: {cells.size} cells differ, {int((qd[cells] < 0).sum())} not split along a diagonal",
              flush=True)
        np.savez_compressed(path, **out)


def ellipse():
    sys.path.insert(0, MG.REF)
    import EllipseRaytrace3D as E
    num = 317
    source = np.zeros((3, num * num))
    l1h, l2h, inc_h, mlen_h = np.float64(146.), np.float64(0.086), np.float64(0.214), np.float64(0.060)
    inc_h /= 20
    ell_v = E.ell(l1h, l2h, inc_h, mlen_h)
    angle_y = np.linspace(ell_v.sita1_1, ell_v.sita1_2, num)
    angle_z = np.linspace(-np.pi / 2 + 1e-9, np.pi / 2 - 1e-9, num)
    angle_z -= np.mean(angle_z)
    YY, ZZ = np.meshgrid(angle_y, angle_z)
    vec = np.zeros((3, num, num))
    vec[0] = 1
    vec[1] = np.tan(YY)
    vec[2] = np.tan(ZZ)
    vec = E.normalize_vector(vec.reshape(3, -1))
    ell_v.coeffs("y")
    ell_v.calc_reflect(vec, source)
    focus = E.PlanePoints(ell_v.dist_s_f, 1e-8, ell_v.reflect, ell_v.points)
    np.savez_compressed(
        os.path.join(MG.OUT, "ellipse_317.npz"), coeffs=np.array(ell_v.coeffs), dir=vec, points=ell_v.points,
        normal=ell_v.N_ell, reflect=ell_v.reflect, plane_pos=ell_v.dist_s_f, plane_delta=1e-8,
        det0=focus.points0, det1=focus.points1, det2=focus.points2,
    )
    print("ellipse_317 written", flush=True)


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "psf"
    if what == "ellipse":
        ellipse()
        return
    A = _import_akb()
    if what == "psf":
        psf(A)
    elif what == "qhull":
        qhull(A, [int(a) for a in sys.argv[2:]] or [1001, 3163])
    else:
        raise SystemExit(f"unknown fixture {what!r}")


if __name__ == "__main__":
    main()
