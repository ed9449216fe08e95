"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

Run in the build container only (the reference is read from /root/reference and never travels):

    python tests/golden/make_golden.py

The reference (Kakekakechan/AKBRaytracing) has no tests and ships no fixtures,
so every vector here is produced by importing its scripts and recording what its own functions
return. Imports need three stand-ins for modules the container lacks and the recorded paths do
not use: numba (njit = identity, prange = range; AKB_raytrace_20250312.py:19-20 imports it
without using it; Wavecalc_raytrace_fromData_CPU0402.py:71 decorates compute_u_parallel), and
cv2 / tifffile (only reached after the recorded quantities, AKB_raytrace_20250312.py:3693, :3731).

Recorded (numpy 2.2, scipy 1.15, float64):
  akb_geometry.json          4-mirror Wolter III+I geometry of plot_result_debug (Setting12 /
                             setting11, :1706-1755) at the __main__ best-alignment params (:14586),
                             option_set=True: the four quadrics in trace order, root signs,
                             detector planes, ray-grid angle endpoints and offsets.
  kb_geometry.json           same for KB_debug defaults (:9942), params = 0.
  akb_primitives_33.npz      every 1089-ray primitive call of a 33x33 'wave' trace: inputs, outputs.
  akb_raywave_65.npz         65x65 'ray_wave': pass-2 tables, rotated hit/direction, detcenter,
                             detcenter2, DistError2 and Wave2 (the griddata inputs, :3689).
  akb_psf_65.npz             the compute_psf_fft call of that 'ray_wave' run (66x66 pupil, pad 16):
                             inputs + a crop of the PSF around its peak + axes.
  kb_wave_65.npz             KB_debug 'wave' 65x65: primitive outputs of pass 2 + detector.
  ellipse_33.npz             EllipseRaytrace3D single ellipse (its __main__ geometry, :309-363)
                             33x33 rays: calc_reflect + PlanePoints outputs.
  psf_cases.npz              compute_psf_fft on small synthetic pupils (even/odd, pad, hann,
                             return_efield, pupil_dy_m).
  huygens_cases.npz          forward_propagation_numpy_batch (compute_u_parallel) on real mirror
                             points of the 65x65 AKB trace -> 64 image-grid targets, and a random box.
  legendre_cases.npz         legendre_fit.aberration_legendre_component basis (nx+ny < 5) on 65x65
                             and match_legendre_multi coefficients of the 65x65 Wave2 map stand-in.
"""
import json
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

os.environ.setdefault("MPLBACKEND", "Agg")


def _stub_modules():
    nb = types.ModuleType("numba")

    def njit(*a, **k):
        if a and callable(a[0]):
            return a[0]
        return lambda f: f

    nb.njit = njit
    nb.prange = range
    sys.modules["numba"] = nb
    for name in ("cv2", "tifffile", "h5py"):
        sys.modules[name] = types.ModuleType(name)


class Recorder:
    """Wraps the reference's module-level primitives (they are resolved via globals at call
    time) and records every call."""

    NAMES = ("mirr_ray_intersection", "norm_vector", "reflect_ray", "plane_ray_intersection")

    def __init__(self, mod):
        self.mod = mod
        self.calls = []
        self.orig = {n: getattr(mod, n) for n in self.NAMES}
        for n in self.NAMES:
            setattr(mod, n, self._wrap(n, self.orig[n]))

    def _wrap(self, name, f):
        def g(*a, **k):
            r = f(*a, **k)
            self.calls.append((name, [np.array(x, dtype=np.float64) if not isinstance(x, (bool,)) else x
                                      for x in a], dict(k), np.array(r)))
            return r
        return g

    def restore(self):
        for n, f in self.orig.items():
            setattr(self.mod, n, f)


def best_params():
    # AKB_raytrace_20250312.py:14586-14592 (float64, the live __main__ path)
    p = np.zeros(26)
    p[0] = -5.73452570e-03
    p[1] = -2.87624337e-03
    p[8] = 1.05000000e-02
    p[9] = -3.59399021e-05
    p[13] = 2.39536993e-06
    p[20] = 1.05000000e-02
    p[21] = -3.59399021e-05
    p[25] = 2.39536993e-06
    return p


def run_akb(A, n, option, record_tan=False):
    A.wave_num_H = n
    A.wave_num_V = n
    A.option_set = True
    rec = Recorder(A)
    grid_calls = []
    psf_calls = []
    orig_grid = A.griddata
    orig_psf = A.compute_psf_fft

    def griddata(points, values, xi, method="linear", **kw):
        grid_calls.append((np.array(points[0]), np.array(points[1]), np.array(values)))
        return orig_grid(points, values, xi, method=method, **kw)

    def psf(opd, amp, wl, dx, f, pad_factor=2, window=None, return_efield=False, pupil_dy_m=None):
        r = orig_psf(opd, amp, wl, dx, f, pad_factor=pad_factor, window=window,
                     return_efield=return_efield, pupil_dy_m=pupil_dy_m)
        psf_calls.append(dict(opd=np.array(opd), amp=np.array(amp), wl=wl, dx=dx, f=f, pad=pad_factor,
                              dy=pupil_dy_m, out=r))
        return r

    A.griddata = griddata
    A.compute_psf_fft = psf
    tan_log, lin_log = [], []
    orig_tan, orig_lin = np.tan, np.linspace
    if record_tan:
        def tan(x, *a, **k):
            r = orig_tan(x, *a, **k)
            tan_log.append((np.array(x), np.array(r)))
            return r

        def linspace(start, stop, num=50, *a, **k):
            r = orig_lin(start, stop, num, *a, **k)
            lin_log.append((float(start), float(stop), int(num)))
            return r
        np.tan = tan
        np.linspace = linspace
    result = None
    err = None
    try:
        result = A.plot_result_debug(best_params(), option, option_save=False)
    except Exception as e:  # cv2 stand-in reached after the recorded quantities
        err = repr(e)
    finally:
        np.tan, np.linspace = orig_tan, orig_lin
        A.griddata = orig_grid
        A.compute_psf_fft = orig_psf
        rec.restore()
    return rec.calls, grid_calls, psf_calls, tan_log, lin_log, result, err


def big(calls, n):
    return [c for c in calls if c[3].ndim == 2 and c[3].shape[1] == n]


def main():
    _stub_modules()
    sys.path.insert(0, REF)
    work = tempfile.mkdtemp(prefix="akb_golden_")
    os.chdir(work)  # the reference creates output folders in CWD at import (:102-114)
    import AKB_raytrace_20250312 as A
    import EllipseRaytrace3D as E
    import legendre_fit as lf
    import psf_fft
    import Wavecalc_raytrace_fromData_CPU0402 as W
    import matplotlib.pyplot as plt

    meta = {"numpy": np.__version__, "reference": "Kakekakechan/AKBRaytracing @ /root/reference"}
    import scipy
    meta["scipy"] = scipy.__version__

    # ------------------------------------------------------------------ AKB geometry (65 ray grid)
    n = 65
    calls, grid_calls, psf_calls, tan_log, lin_log, _, err = run_akb(A, n, "ray_wave", record_tan=True)
    print("ray_wave stopped at:", err)
    plt.close("all")
    N = n * n
    bc = big(calls, N)
    isects = [c for c in bc if c[0] == "mirr_ray_intersection"]
    planes = [c for c in bc if c[0] == "plane_ray_intersection"]
    assert len(isects) == 8, len(isects)
    mirrors = [dict(coeffs=[float(x) for x in c[1][0]], negative=bool(c[2].get("negative", False)))
               for c in isects[:4]]
    for a, b in zip(isects[:4], isects[4:]):
        assert np.array_equal(a[1][0], b[1][0])
    det1 = [float(x) for x in planes[0][1][0]]
    # tan tables of pass 1: the first array call of length n is tan(rand_p0h); the scalar calls
    # that follow are tan(rand_p0v[i]) for the n rows (:2711-2715)
    arr_calls = [i for i, (x, r) in enumerate(tan_log) if x.ndim == 1 and x.size == n]
    first = arr_calls[0]
    rand_h = tan_log[first][0]
    rand_v = np.array([tan_log[first + 1 + 2 * i][0] for i in range(n)], dtype=np.float64)
    tan_h = tan_log[first][1]
    tan_v = np.array([tan_log[first + 1 + 2 * i][1] for i in range(n)], dtype=np.float64)
    lins = [l for l in lin_log if l[2] == n]
    lh, lv = lins[0], lins[1]
    theta1_h = np.float64(0.000145746388538841)  # setting11, :1738
    theta1_v = np.float64(5.55983241203018E-05)   # Setting12, :1712
    assert np.array_equal(np.linspace(lh[0], lh[1], n) - theta1_h, rand_h)
    assert np.array_equal(np.linspace(lv[0], lv[1], n) - theta1_v, rand_v)
    # the ray_wave detector 2 plane (:3618-3621) is the second plane call after the tilt
    det2 = [float(x) for x in planes[-1][1][0]]
    geom = dict(
        name="AKB Wolter III+I Setting12/setting11 best alignment (AKB_raytrace_20250312.py:1706-1755, :14586)",
        mirrors=mirrors, det1=det1, det2=det2,
        angle_h=dict(start=lh[0], stop=lh[1], offset=float(theta1_h)),
        angle_v=dict(start=lv[0], stop=lv[1], offset=float(theta1_v)),
        source=[0.0, 0.0, 0.0], wavelength_m=13.5e-9, defocus_wave_m=1e-2,
        meta=meta,
    )
    with open(os.path.join(OUT, "akb_geometry.json"), "w") as f:
        json.dump(geom, f, indent=1)

    # ray_wave outputs
    (d2y, d2z, dist_err2), (_, _, wave2) = grid_calls[0], grid_calls[1]
    det_after = planes[-2]
    det2c = planes[-1]
    np.savez_compressed(
        os.path.join(OUT, "akb_raywave_65.npz"),
        tan_h=tan_h, tan_v=tan_v, rand_h=rand_h, rand_v=rand_v,
        pass1_dir=isects[0][1][1], pass2_dir=isects[4][1][1],
        pass2_hits=np.stack([c[3] for c in isects[4:]]),
        rot_dir=det_after[1][1], rot_pt=det_after[1][2],
        detcenter=det_after[3], detcenter2=det2c[3],
        dist_err2=dist_err2, wave2=wave2, det2_y=d2y, det2_z=d2z,
    )
    # compute_psf_fft call made by psf_calc (:1200)
    pc = psf_calls[0]
    psf_img, x_im, y_im = pc["out"]
    iy, ix = np.unravel_index(np.argmax(psf_img), psf_img.shape)
    h = 48
    np.savez_compressed(
        os.path.join(OUT, "akb_psf_65.npz"),
        opd=pc["opd"], amp=pc["amp"], wl=pc["wl"], dx=pc["dx"], dy=pc["dy"], f=pc["f"], pad=pc["pad"],
        crop=psf_img[iy - h:iy + h, ix - h:ix + h], crop_origin=np.array([iy - h, ix - h]),
        shape=np.array(psf_img.shape), x_im=x_im, y_im=y_im, psf_sum=np.sum(psf_img),
    )

    # ------------------------------------------------------------------ primitive I/O at 33x33
    n33 = 33
    calls33, _, _, _, _, wave_ret, _ = run_akb(A, n33, "wave")
    plt.close("all")
    prim = {}
    for idx, (name, args, kw, out) in enumerate(big(calls33, n33 * n33)):
        key = f"c{idx:02d}_{name}"
        for j, a in enumerate(args):
            prim[f"{key}_in{j}"] = a
        prim[f"{key}_neg"] = np.array(bool(kw.get("negative", False)))
        prim[f"{key}_out"] = out
    np.savez_compressed(os.path.join(OUT, "akb_primitives_33.npz"), **prim)

    # ------------------------------------------------------------------ KB 'wave' 65x65
    A.wave_num_H = 65
    A.wave_num_V = 65
    recK = Recorder(A)
    tanK, linK = [], []
    orig_tan, orig_lin = np.tan, np.linspace

    def tanr(x, *a, **k):
        r = orig_tan(x, *a, **k)
        tanK.append((np.array(x), np.array(r)))
        return r

    def linr(start, stop, num=50, *a, **k):
        r = orig_lin(start, stop, num, *a, **k)
        linK.append((float(start), float(stop), int(num)))
        return r
    np.tan, np.linspace = tanr, linr
    try:
        A.KB_debug(np.zeros(26), 1, 1, "wave", option_save=False)
    except Exception as e:
        print("KB_debug stopped:", repr(e))
    finally:
        np.tan, np.linspace = orig_tan, orig_lin
        recK.restore()
    plt.close("all")
    kb_big = big(recK.calls, 65 * 65)
    kb_isect = [c for c in kb_big if c[0] == "mirr_ray_intersection"]
    kb_plane = [c for c in kb_big if c[0] == "plane_ray_intersection"]
    first = [i for i, (x, r) in enumerate(tanK) if x.ndim == 1 and x.size == 65][0]
    krand_h = tanK[first][0]
    krand_v = np.array([tanK[first + 1 + 2 * i][0] for i in range(65)])
    klins = [l for l in linK if l[2] == 65]
    klh, klv = klins[0], klins[1]
    # KB_debug centres the angles on the mean of the two edge angles (:10955-10956); with no
    # source shift those are exactly the linspace endpoints
    off_h = float(np.mean([klh[0], klh[1]]))
    off_v = float(np.mean([klv[0], klv[1]]))
    assert np.array_equal(np.linspace(klh[0], klh[1], 65) - off_h, krand_h)
    assert np.array_equal(np.linspace(klv[0], klv[1], 65) - off_v, krand_v)
    kb_geom = dict(
        name="KB_debug EUV HighNA defaults (AKB_raytrace_20250312.py:9942), params = 0",
        mirrors=[dict(coeffs=[float(x) for x in c[1][0]], negative=bool(c[2].get("negative", False)))
                 for c in kb_isect[:2]],
        det1=[float(x) for x in kb_plane[0][1][0]],
        angle_h=dict(start=klh[0], stop=klh[1], offset=off_h),
        angle_v=dict(start=klv[0], stop=klv[1], offset=off_v),
        source=[0.0, 0.0, 0.0], meta=meta)
    with open(os.path.join(OUT, "kb_geometry.json"), "w") as f:
        json.dump(kb_geom, f, indent=1)
    kb_refl = [c for c in kb_big if c[0] == "reflect_ray"]
    np.savez_compressed(
        os.path.join(OUT, "kb_wave_65.npz"),
        pass1_dir=kb_isect[0][1][1], pass1_hits=np.stack([c[3] for c in kb_isect[:2]]),
        pass1_refl=kb_refl[1][3],
        pass2_dir=kb_isect[2][1][1], pass2_hits=np.stack([c[3] for c in kb_isect[2:4]]),
        pass2_refl=kb_refl[3][3], pass2_det=kb_plane[1][3],
    )

    # ------------------------------------------------------------------ EllipseRaytrace3D (C1)
    num = 33
    source = np.zeros((3, num * num))
    l1h, l2h, inc_h, mlen_h, wd_v, inc_v, mlen_v = [np.float64(146.), np.float64(0.086), np.float64(0.214),
                                                    np.float64(0.060), np.float64(0.0211), np.float64(0.21),
                                                    np.float64(0.0232)]
    inc_h /= 20
    inc_v /= 20
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
    focus = E.PlanePoints(ell_v.dist_s_f, 1e-9, ell_v.reflect, ell_v.points)
    np.savez_compressed(
        os.path.join(OUT, "ellipse_33.npz"), coeffs=np.array(ell_v.coeffs), dir=vec, points=ell_v.points,
        normal=ell_v.N_ell, reflect=ell_v.reflect, plane_pos=ell_v.dist_s_f, plane_delta=1e-9,
        det0=focus.points0, det1=focus.points1, det2=focus.points2,
    )

    # ------------------------------------------------------------------ compute_psf_fft cases
    rng = np.random.default_rng(7)
    cases = {}
    specs = [(32, 32, 4, None, False, None), (31, 33, 2, "hann", True, None),
             (16, 24, 1, None, True, 3e-6), (20, 20, 3, "hann", False, 2e-6), (9, 7, 5, None, False, None)]
    for k, (ny, nx, pad, win, eff, dy) in enumerate(specs):
        yy, xx = np.mgrid[0:ny, 0:nx]
        r2 = ((yy - ny / 2) / (ny / 2)) ** 2 + ((xx - nx / 2) / (nx / 2)) ** 2
        amp = (r2 <= 1.0).astype(float)
        opd = 2e-9 * rng.standard_normal((ny, nx))
        opd[0, 0] = np.nan
        amp[1, 1] = np.nan
        out = psf_fft.compute_psf_fft(opd, amp, 13.5e-9, 5e-6, 1e-2, pad_factor=pad, window=win,
                                      return_efield=eff, pupil_dy_m=dy)
        cases[f"k{k}_opd"] = opd
        cases[f"k{k}_amp"] = amp
        cases[f"k{k}_spec"] = np.array([ny, nx, pad, 1 if win else 0, 1 if eff else 0, dy if dy else -1.0])
        cases[f"k{k}_psf"] = out[0]
        cases[f"k{k}_x"] = out[1]
        cases[f"k{k}_y"] = out[2]
        if eff:
            cases[f"k{k}_efield"] = out[3]
    np.savez_compressed(os.path.join(OUT, "psf_cases.npz"), **cases)

    # ------------------------------------------------------------------ Huygens
    # sources: the V-hyperboloid hit points of the 65x65 AKB pass 2 with a synthetic dS and field;
    # targets: an 8x8 grid around the focus.
    pts = np.load(os.path.join(OUT, "akb_raywave_65.npz"))["pass2_hits"][0]
    M = pts.shape[1]
    ds = np.full(M, 1e-10) * (1.0 + 0.1 * rng.random(M))
    u_back = np.exp(1j * rng.random(M)) * (1.0 + 0.05 * rng.standard_normal(M))
    foc = np.load(os.path.join(OUT, "akb_raywave_65.npz"))["detcenter"].mean(axis=1)
    gy, gz = np.meshgrid(np.linspace(-2e-7, 2e-7, 8), np.linspace(-2e-7, 2e-7, 8))
    tx = np.full(64, foc[0])
    ty = foc[1] + gy.ravel()
    tz = foc[2] + gz.ravel()
    k = 2.0 * np.pi / np.float64(13.5e-9)
    u1 = W.forward_propagation_numpy_batch(tx, ty, tz, pts[0], pts[1], pts[2], u_back, k, ds)
    # random box
    M2, N2 = 3000, 50
    sx, sy, sz = rng.random(M2) * 1e-3, rng.random(M2) * 1e-3, rng.random(M2) * 1e-3
    ux = rng.random(N2) * 1e-3
    uy = rng.random(N2) * 1e-3
    uz = 0.1 + rng.random(N2) * 1e-3
    ub2 = rng.standard_normal(M2) + 1j * rng.standard_normal(M2)
    ds2 = rng.random(M2)
    k2 = 2.0 * np.pi / np.float64(1.35e-9)
    u2 = W.forward_propagation_numpy_batch(ux, uy, uz, sx, sy, sz, ub2, k2, ds2)
    np.savez_compressed(os.path.join(OUT, "huygens_cases.npz"),
                        a_tx=tx, a_ty=ty, a_tz=tz, a_sx=pts[0], a_sy=pts[1], a_sz=pts[2], a_u=u_back,
                        a_ds=ds, a_k=k, a_out=u1,
                        b_tx=ux, b_ty=uy, b_tz=uz, b_sx=sx, b_sy=sy, b_sz=sz, b_u=ub2, b_ds=ds2, b_k=k2,
                        b_out=u2)

    # ------------------------------------------------------------------ Legendre basis
    H = 65
    xs = np.linspace(-1, 1, H)
    basis = []
    orders = []
    for i in range(5):          # match_legendre_multi order (legendre_fit.py:82-90)
        for j in range(i + 1):
            nx_, ny_ = j, i - j
            Z = lf.aberration_legendre_component(xs, xs, nx_, ny_)
            basis.append(Z)
            orders.append((ny_, nx_))
    wave_map = np.load(os.path.join(OUT, "akb_raywave_65.npz"))["wave2"].reshape(65, 65)
    fitted, coefs, _names = lf.match_legendre_multi(wave_map, 5)
    np.savez_compressed(os.path.join(OUT, "legendre_cases.npz"), basis=np.array(basis),
                        orders=np.array(orders), wave_map=wave_map, fit=fitted, coefs=np.array(coefs))
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
