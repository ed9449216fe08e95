"""The oracle against vectors recorded from the reference itself (tests/golden/make_golden.py).
CPU only. Bitwise where the reference's arithmetic is IEEE basic operations."""
import numpy as np
import pytest

import oracle as O
import oracle.huygens as OH
import oracle.legendre as OL
import oracle.pipeline as OPL
import oracle.psf as OP
from conftest import golden, golden_json


def _prim_calls():
    d = golden("akb_primitives_33.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files})
    for k in keys:
        name = k.split("_", 1)[1]
        ins = [d[f"{k}_in{j}"] for j in range(3) if f"{k}_in{j}" in d.files]
        yield k, name, ins, bool(d[f"{k}_neg"]), d[f"{k}_out"]


def test_primitives_bitwise_vs_reference():
    n = 0
    for key, name, ins, neg, ref in _prim_calls():
        f = getattr(O, name)
        out = f(*ins, negative=True) if neg else f(*ins)
        assert np.array_equal(out, ref, equal_nan=True), key
        n += 1
    assert n == 28


@pytest.mark.parametrize("fixture", ["ellipse_33.npz", "ellipse_317.npz"])
def test_ellipse_chain_bitwise(fixture):
    """C1 (BASELINE configs[0]) at 33^2 and at its own 317^2: the oracle equals the reference's run."""
    d = golden(fixture)
    src = np.zeros_like(d["dir"])
    pts = O.mirr_ray_intersection(d["coeffs"], d["dir"], src)
    nrm = O.norm_vector(d["coeffs"], pts)
    refl = O.reflect_ray(d["dir"], nrm)
    assert np.array_equal(pts, d["points"])
    assert np.array_equal(nrm, d["normal"])
    assert np.array_equal(refl, d["reflect"])
    pos, delta = float(d["plane_pos"]), float(d["plane_delta"])
    for key, j in (("det0", -pos), ("det1", -pos + delta), ("det2", -pos - delta)):
        c = np.zeros(10)
        c[6], c[9] = 1.0, j
        assert np.array_equal(O.plane_ray_intersection(c, refl, pts), d[key]), key


def test_akb_ray_wave_pipeline_bitwise():
    g = golden_json("akb_geometry.json")
    f = golden("akb_raywave_65.npz")
    r = OPL.akb_ray_wave(g, 65)
    assert np.array_equal(r["tan_h"], f["tan_h"]) and np.array_equal(r["tan_v"], f["tan_v"])
    assert np.array_equal(r["dirs2"], f["pass2_dir"])
    assert np.array_equal(np.stack(r["hits"]), f["pass2_hits"])
    for a, b in (("r4_rot", "rot_dir"), ("p4_rot", "rot_pt"), ("detcenter", "detcenter"),
                 ("detcenter2", "detcenter2"), ("dist_err2", "dist_err2"), ("wave2", "wave2")):
        assert np.array_equal(r[a], f[b], equal_nan=True), a


def test_kb_wave_pipeline_bitwise():
    g = golden_json("kb_geometry.json")
    f = golden("kb_wave_65.npz")
    r = OPL.kb_wave(g, 65)
    assert np.array_equal(np.stack(r["hits1"]), f["pass1_hits"])
    assert np.array_equal(r["dirs2"], f["pass2_dir"])
    assert np.array_equal(np.stack(r["hits2"]), f["pass2_hits"])
    assert np.array_equal(r["refl2"], f["pass2_refl"])
    assert np.array_equal(r["det"], f["pass2_det"])


def test_array_tan_equals_rowwise_tan():
    # the driver takes np.tan of each V angle as a scalar (:2713); the pipelines use one array call
    g = golden_json("akb_geometry.json")
    for n in (65, 1001, 3163):
        v = g["angle_v"]
        r = np.linspace(v["start"], v["stop"], n) - np.float64(v["offset"])
        assert np.array_equal(np.tan(r), np.array([np.tan(x) for x in r]))


@pytest.mark.parametrize("n", [0, 1, 5, 8, 9, 127, 128, 129, 1000, 8191, 8192, 8193, 20000, 100003])
def test_np_sum_restatement(n):
    rng = np.random.default_rng(n)
    x = 146.0 + rng.standard_normal(n) * 1e-3
    s, c = O.np_sum(x)
    assert (s == np.sum(x)) or n == 0
    assert c == n
    if n > 3:
        x[::7] = np.nan
        s, c = O.np_sum(x, nan=True)
        assert s == np.nansum(x)
        assert s / c == np.nanmean(x)


def test_np_sum_axis1_rows():
    rng = np.random.default_rng(3)
    a = rng.standard_normal((3, 50001)) + [[146.0], [0.01], [-0.02]]
    m = np.mean(a, axis=1)
    for r in range(3):
        s, c = O.np_sum(a[r])
        assert s / c == m[r]


def test_psf_restatement_bitwise():
    d = golden("psf_cases.npz")
    for k in range(5):
        ny, nx, pad, win, eff, dy = d[f"k{k}_spec"]
        r = OP.psf(d[f"k{k}_opd"], d[f"k{k}_amp"], 13.5e-9, 5e-6, 1e-2, int(pad), "hann" if win else None,
                   bool(eff), None if dy < 0 else dy)
        assert np.array_equal(r[0], d[f"k{k}_psf"])
        assert np.array_equal(r[1], d[f"k{k}_x"]) and np.array_equal(r[2], d[f"k{k}_y"])
        if eff:
            assert np.array_equal(r[3], d[f"k{k}_efield"])


def test_psf_restatement_real_pupil():
    d = golden("akb_psf_65.npz")
    I, x, y = OP.psf(d["opd"], d["amp"], float(d["wl"]), float(d["dx"]), float(d["f"]), int(d["pad"]),
                     dy=float(d["dy"]))
    assert I.shape == tuple(d["shape"])
    y0, x0 = d["crop_origin"]
    h = d["crop"].shape[0]
    assert np.array_equal(I[y0:y0 + h, x0:x0 + h], d["crop"])
    assert np.array_equal(x, d["x_im"]) and np.array_equal(y, d["y_im"])


def test_huygens_restatement():
    h = golden("huygens_cases.npz")
    for p in "ab":
        o = OH.propagate(h[p + "_tx"], h[p + "_ty"], h[p + "_tz"], h[p + "_sx"], h[p + "_sy"], h[p + "_sz"],
                         h[p + "_u"], h[p + "_k"], h[p + "_ds"])
        assert np.array_equal(o, h[p + "_out"])
        # the C speed baseline (sequential sum order): tolerance
        c = O.huygens_c(h[p + "_tx"], h[p + "_ty"], h[p + "_tz"], h[p + "_sx"], h[p + "_sy"], h[p + "_sz"],
                      h[p + "_u"] * h[p + "_ds"], h[p + "_k"])
        assert np.max(np.abs(c - h[p + "_out"])) <= 1e-9 * np.max(np.abs(h[p + "_out"]))


def test_legendre_basis():
    d = golden("legendre_cases.npz")
    xs = np.linspace(-1, 1, 65)
    B = np.array([OL.component(xs, xs, nx, ny) for ny, nx in OL.orders(5)])
    assert [tuple(o) for o in d["orders"]] == OL.orders(5)
    np.testing.assert_allclose(B, d["basis"], rtol=0, atol=1e-14)
    _, coefs = OL.fit_multi(d["wave_map"], 5)
    # tolerance relative to the largest coefficient (the 65x65 map carries a ~1e7 nm offset)
    np.testing.assert_allclose(coefs, d["coefs"], rtol=0, atol=1e-14 * np.max(np.abs(d["coefs"])))


def test_all_nan_and_passthrough_rules():
    # a ray that misses: the WHOLE output is NaN (ref :457-459)
    c = [1.0, 1.0, 1.0, 0, 0, 0, 0, 0, 0, -1.0]  # unit sphere
    ray = np.array([[1.0, 0.0], [0.0, 1.0], [0.0, 0.0]])
    src = np.array([[-5.0, -5.0], [0.0, 5.0], [0.0, 0.0]])  # 2nd ray passes y=5 parallel to y? misses
    src[:, 1] = [5.0, 5.0, 0.0]
    out = O.mirr_ray_intersection(c, ray, src)
    assert np.isnan(out).all()
    # a zero vector: normalize_vector returns its input unchanged (ref :530-532)
    v = np.array([[0.0, 1.0], [0.0, 2.0], [0.0, 2.0]])
    assert O.normalize_vector(v) is v


def test_oracle_rotate_matches_scipy_fixtures():
    """oracle/psfcalc.rotate restates scipy.ndimage.rotate(order 3, constant, reshape False)."""
    import oracle.psfcalc as PC
    d = golden("scipy_rotate.npz")
    for k in range(4):
        ang = float(d[f"k{k}_angle"])
        assert np.max(np.abs(PC.rotate(d[f"k{k}_in"], ang) - d[f"k{k}_out"])) <= 1e-13
        assert np.max(np.abs(PC.rotate(d[f"k{k}_mask"], ang) - d[f"k{k}_mask_out"])) <= 1e-13


def test_oracle_psf_calc_matches_reference():
    """psf_calc of the reference's 65x65 ray_wave run: rotation estimate (exact), the rotated
    map it handed compute_psf_fft (NaN pattern exact, values to 1e-15 nm) and the trimmed PSF."""
    import oracle.psfcalc as PC
    f = golden("akb_psfcalc_65.npz")
    r = PC.psf_calc(f["psf_calc_in"], f["grid_H"], f["grid_V"], float(f["defocus"]))
    assert r["rot"] == f["rot"]
    assert np.array_equal(np.isnan(r["rotated"]), np.isnan(f["rotated"]))
    assert np.nanmax(np.abs(r["rotated"] - f["rotated"])) <= 1e-15
    assert r["psf_trimmed"].shape == f["psf_trimmed"].shape
    assert np.max(np.abs(r["psf_trimmed"] - f["psf_trimmed"])) <= 1e-12
    assert np.array_equal(r["x_im"], f["x_im"])


@pytest.mark.parametrize("n", [1001, 3163])
def test_oracle_psf_calc_full_size_matches_reference(n):
    """psf_calc at the bench's sizes: the reference's own call on its own plane-corrected 128^2 map
    of the n^2 trace (akb_psf_full.npz, make_golden_full_extra.py psf): rotation estimate exact, the
    rotated map to 1e-15 nm, the trimmed 2048^2 PSF to 1e-12 of its peak."""
    import oracle.psfcalc as PC
    full = golden("akb_raywave_full.npz")
    f = golden("akb_psf_full.npz")
    GH, GV = np.meshgrid(full[f"n{n}_gx"], full[f"n{n}_gy"])
    r = PC.psf_calc(full[f"n{n}_map_wave_c"], GH - np.mean(GH), GV - np.mean(GV), 1e-2)
    assert r["rot"] == f[f"n{n}_rot"]
    assert np.array_equal(np.isnan(r["rotated"]), np.isnan(f[f"n{n}_rotated"]))
    assert np.nanmax(np.abs(r["rotated"] - f[f"n{n}_rotated"])) <= 1e-15 * max(1.0, np.nanmax(np.abs(r["rotated"])))
    assert r["psf_trimmed"].shape == f[f"n{n}_psf_crop"].shape
    assert np.max(np.abs(r["psf_trimmed"] - f[f"n{n}_psf_crop"])) <= 1e-12
    assert np.array_equal(r["x_im"], f[f"n{n}_x_im"]) and np.array_equal(r["y_im"], f[f"n{n}_y_im"])


def test_oracle_calc_ds_matches_reference():
    """calc_dS on the four mirror grids of the reference's 65x65 run, bit for bit."""
    f = golden("akb_raywave_65.npz")
    d = golden("wavedata_65.npz")
    for k in range(4):
        assert np.array_equal(O.calc_dS(f["pass2_hits"][k], 65, 65), d["ds"][k])


def test_plane_correction_oracle_vs_reference():
    """oracle/pupilmap restates plane_correction_with_nan_and_outlier_filter (:9630) as lstsq;
    the reference's own curve_fit output on its 65x65 ray_wave map pins it."""
    import oracle.pupilmap as PM
    f = golden("akb_psfcalc_65.npz")
    got = PM.plane_correction_with_nan_and_outlier_filter(f["plane_in"])
    want = f["plane_out"]
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.nanmax(np.abs(got - want)) <= 1e-12 * (np.nanmax(want) - np.nanmin(want))
