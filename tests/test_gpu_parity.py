"""HIP path vs the reference's recorded vectors and vs the oracle (run on an MI355X).

Bar: bit-exact for the trace primitives, the fused chain, the numpy-order sums and everything
the tilt step does not touch. After the tilt the per-ray arctan of the exit slopes comes from
OCML atan instead of glibc atan, so the tilt angles may differ by an ulp: rotated quantities are
held to a few ulp and the OPD to 1e-4 nm absolute. PSF intensity and Huygens
fields: 1e-6 relative to the peak / max magnitude (BASELINE.json north_star), observed ~1e-12.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O
import oracle.pipeline as OPL
from conftest import ROOT, golden, golden_json

pytestmark = pytest.mark.gpu


def _ulp_diff(a, b):
    """max |a - b| in ulps of the largest magnitude of each row (so components near zero are
    judged on the scale of the vector they belong to)."""
    a = np.atleast_2d(np.asarray(a, dtype=np.float64))
    b = np.atleast_2d(np.asarray(b, dtype=np.float64))
    worst = 0.0
    for ra, rb in zip(a, b):
        ok = ~(np.isnan(ra) & np.isnan(rb))
        if not ok.any():
            continue
        scale = np.spacing(np.max(np.abs(rb[ok])))
        worst = max(worst, float(np.max(np.abs(ra[ok] - rb[ok])) / scale))
    return worst


# ----------------------------------------------------------------------------- primitives

def test_primitives_bitwise_vs_reference(gpu):
    from akbraytracing_amd import primitives as P
    d = golden("akb_primitives_33.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files})
    for k in keys:
        name = k.split("_", 1)[1]
        ins = [d[f"{k}_in{j}"] for j in range(3) if f"{k}_in{j}" in d.files]
        f = getattr(P, name)
        out = f(*ins, negative=True) if bool(d[f"{k}_neg"]) else f(*ins)
        assert isinstance(out, np.ndarray)
        assert np.array_equal(out, d[f"{k}_out"], equal_nan=True), k


def test_small_and_broadcast_calls(gpu):
    """The drivers' N = 1..4 centre/edge-ray calls and (3,) ray broadcasting (:1909, :2252, :2828)."""
    from akbraytracing_amd import primitives as P
    g = golden_json("akb_geometry.json")
    c = g["mirrors"][0]["coeffs"]
    th = 5.55983241203018e-05
    ray = np.array([[np.cos(th)], [0.0], [np.sin(th)]])
    src = np.zeros((3, 1))
    assert np.array_equal(P.mirr_ray_intersection(c, ray, src), O.mirr_ray_intersection(c, ray, src))
    rng = np.random.default_rng(0)
    dirs = O.normalize_vector(np.vstack([np.ones(4), rng.normal(0, 1e-4, 4), rng.normal(0, 1e-4, 4)]))
    src4 = np.zeros((3, 4))
    p_gpu = P.mirr_ray_intersection(c, dirs, src4)
    assert np.array_equal(p_gpu, O.mirr_ray_intersection(c, dirs, src4))
    ray1d = dirs[:, 0].copy()
    assert np.array_equal(P.mirr_ray_intersection(c, ray1d, src4), O.mirr_ray_intersection(c, ray1d, src4))
    nv = P.norm_vector(c, p_gpu)
    assert np.array_equal(nv, O.norm_vector(c, p_gpu))
    assert np.array_equal(P.reflect_ray(dirs, nv), O.reflect_ray(dirs, nv))
    with pytest.raises(ValueError):
        P.mirr_ray_intersection(c, dirs, src)  # (3,4) rays into a (3,1) source: numpy raises too


def test_value_rules(gpu):
    from akbraytracing_amd import primitives as P
    sphere = [1.0, 1.0, 1.0, 0, 0, 0, 0, 0, 0, -1.0]
    ray = np.array([[1.0, 1.0], [0.0, 0.0], [0.0, 0.0]])
    src = np.array([[-5.0, -5.0], [0.0, 5.0], [0.0, 0.0]])
    out = P.mirr_ray_intersection(sphere, ray, src)
    assert out.shape == (3, 2) and np.isnan(out).all()
    v = np.array([[0.0, 1.0], [0.0, 2.0], [0.0, 2.0]])
    assert P.normalize_vector(v) is v
    # zero gradient at the origin of a sphere: norm_vector passes the raw gradient through
    pt = np.array([[0.0, 0.5], [0.0, 0.0], [0.0, 0.0]])
    assert np.array_equal(P.norm_vector(sphere, pt), O.norm_vector(sphere, pt))
    # parallel plane: per-ray inf/NaN, not all-NaN
    c = np.zeros(10)
    c[6], c[9] = 1.0, -1.0
    r = np.array([[0.0, 1.0], [1.0, 0.0], [0.0, 0.0]])
    s = np.zeros((3, 2))
    got = P.plane_ray_intersection(c, r, s)
    with np.errstate(all="ignore"):
        ref = O.plane_ray_intersection(c, r, s)
    assert np.array_equal(got, ref, equal_nan=True)


def test_torch_inputs_stay_on_device(gpu):
    from akbraytracing_amd import primitives as P
    d = golden("akb_primitives_33.npz")
    c = d["c00_mirr_ray_intersection_in0"]
    ray = torch.from_numpy(d["c00_mirr_ray_intersection_in1"]).to(gpu)
    src = torch.from_numpy(d["c00_mirr_ray_intersection_in2"]).to(gpu)
    out = P.mirr_ray_intersection(c, ray, src)
    assert isinstance(out, torch.Tensor) and out.is_cuda
    assert np.array_equal(out.cpu().numpy(), d["c00_mirr_ray_intersection_out"])


@pytest.mark.parametrize("fixture", ["ellipse_33.npz", "ellipse_317.npz"])
def test_ellipse_config1(gpu, fixture):
    """BASELINE configs[0] (C1): EllipseRaytrace3D's __main__ ellipse - calc_reflect and the three
    PlanePoints planes (position, position -+ delta, EllipseRaytrace3D.py:241-262) - bit for bit vs
    the reference's own run, at 33^2 and at C1's own 317^2 (1.0e5 rays)."""
    from akbraytracing_amd import primitives as P
    d = golden(fixture)
    src = np.zeros_like(d["dir"])
    pts = P.mirr_ray_intersection(d["coeffs"], d["dir"], src)
    nrm = P.norm_vector(d["coeffs"], pts)
    refl = P.reflect_ray(d["dir"], nrm)
    assert np.array_equal(pts, d["points"]) and np.array_equal(refl, d["reflect"])
    assert np.array_equal(nrm, d["normal"])
    pos, delta = float(d["plane_pos"]), float(d["plane_delta"])
    for key, c9 in (("det0", -pos), ("det1", -pos + delta), ("det2", -pos - delta)):
        c = np.zeros(10)
        c[6], c[9] = 1.0, c9
        assert np.array_equal(P.plane_ray_intersection(c, refl, pts), d[key]), key


def test_rotations_match_reference_blas_order(gpu):
    from akbraytracing_amd import primitives as P
    f = golden("akb_raywave_65.npz")
    r = OPL.akb_ray_wave(golden_json("akb_geometry.json"), 65)
    got_dir = P.rotate_vectors(r["r4"], -r["theta_y"], -r["theta_z"])
    got_pt = P.rotate_points(r["hits"][-1], r["focus_apprx"], -r["theta_y"], -r["theta_z"])
    assert np.array_equal(got_dir, f["rot_dir"])
    assert np.array_equal(got_pt, f["rot_pt"])


def test_arith_shortcuts_bitwise(gpu):
    """The chain kernels' rescale-free sqrt, shared-reciprocal divisions and fused norm/reciprocal
    equal sqrt(), a / b and 1 / sqrt() bit for bit (sign of zero included) over a wide range, and
    fall back to them outside it."""
    from akbraytracing_amd import _lib, device as D
    rng = np.random.default_rng(11)
    n = 4_000_000
    e = rng.integers(-760, 900, n).astype(np.float64)
    a = rng.random(n) * 2.0 ** e
    a[::3] *= -1.0
    b = (rng.random(n) + 0.5) * 2.0 ** rng.integers(-40, 40, n)
    # norms at the edges of the fast path's range, all-ones and one-bit mantissas near 1
    m = 200_000
    edge_e = rng.choice(np.array([-768, -767, -766, -700, -2, -1, 0, 1, 998, 999, 1000]), m).astype(np.float64)
    edge = (1.0 + rng.random(m)) * 2.0 ** edge_e
    ones = np.array([np.nextafter(2.0 ** k, 0.0) for k in range(-300, 300)])
    a = np.concatenate([a, np.sqrt(edge / 3.0), ones, 1.0 + ones])
    b = np.concatenate([b, np.sqrt(edge / 3.0), ones, 1.0 + ones])
    special = np.array([0.0, -0.0, 1.0, 4.0, np.inf, -1.0, np.nan, 1e-300, 5e-324, 2.0 ** -767, 1e305])
    a = np.concatenate([a, special])
    b = np.concatenate([b, np.full(special.shape, 3.0)])
    ta, tb = torch.from_numpy(a).to(gpu), torch.from_numpy(b).to(gpu)
    cols = 13
    out = torch.empty((a.shape[0], cols), dtype=torch.float64, device=gpu)
    _lib.check(_lib.lib().akb_selftest_arith_f64(D.ptr(ta), D.ptr(tb), a.shape[0], D.ptr(out), D.stream_handle()))
    o = out.cpu().numpy()
    bits = lambda v: v.view(np.uint64)
    nan0 = np.isnan(o[:, 1])
    assert np.array_equal(bits(o[~nan0, 0]), bits(o[~nan0, 1])) and np.isnan(o[nan0, 0]).all()
    assert np.array_equal(o[:, 0], np.sqrt(a), equal_nan=True)
    fin = np.isfinite(a)
    assert np.array_equal(bits(o[fin, 2]), bits(o[fin, 3]))
    assert np.array_equal(bits(o[fin, 3]), bits((a / b)[fin]))
    assert np.array_equal(bits(o[fin, 4]), bits(o[fin, 3]))          # positive divisors only
    v = a * a + b * b + b * b
    ok = np.isfinite(v) & (v > 0)
    assert np.array_equal(bits(o[ok, 5]), bits(o[ok, 7]))
    assert np.array_equal(bits(o[ok, 6]), bits(o[ok, 8]))
    assert np.array_equal(bits(o[ok, 8]), bits(1.0 / np.sqrt(v[ok])))
    # the trace's division (core in [2^-300, 2^300], library outside) equals a / b and 1 / b
    with np.errstate(all="ignore"):
        assert np.array_equal(o[:, 11], a / b, equal_nan=True) and np.array_equal(bits(o[fin, 11]), bits((a / b)[fin]))
        assert np.array_equal(bits(o[:, 12]), bits(1.0 / b))
    # and over the whole exponent range, signs, zeros, infinities and NaN, as both operands
    n2 = 2_000_000
    a2 = (rng.random(n2) + 0.5) * 2.0 ** rng.integers(-1074, 1023, n2).astype(np.float64)
    b2 = (rng.random(n2) + 0.5) * 2.0 ** rng.integers(-1074, 1023, n2).astype(np.float64)
    a2[::2] *= -1.0
    b2[::3] *= -1.0
    mid = rng.random(n2) < 0.5  # half inside the core's range, near its edges
    a2[mid] = (rng.random(mid.sum()) + 0.5) * 2.0 ** rng.integers(-302, 302, mid.sum()).astype(np.float64)
    b2[mid] = (rng.random(mid.sum()) + 0.5) * 2.0 ** rng.integers(-302, 302, mid.sum()).astype(np.float64)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 2.0 ** -300, 2.0 ** 300, 1.0, -1.0])
    a2 = np.concatenate([a2, np.repeat(sp, sp.size)])
    b2 = np.concatenate([b2, np.tile(sp, sp.size)])
    t2a, t2b = torch.from_numpy(a2).to(gpu), torch.from_numpy(b2).to(gpu)
    out2 = torch.empty((a2.shape[0], cols), dtype=torch.float64, device=gpu)
    _lib.check(_lib.lib().akb_selftest_arith_f64(D.ptr(t2a), D.ptr(t2b), a2.shape[0], D.ptr(out2), D.stream_handle()))
    o2 = out2.cpu().numpy()
    with np.errstate(all="ignore"):
        q = a2 / b2
        nanq = np.isnan(q)
        assert np.array_equal(np.isnan(o2[:, 11]), nanq) and np.array_equal(bits(o2[~nanq, 11]), bits(q[~nanq]))
        r = 1.0 / b2
        nanr = np.isnan(r)
        assert np.array_equal(np.isnan(o2[:, 12]), nanr) and np.array_equal(bits(o2[~nanr, 12]), bits(r[~nanr]))
    # slope arctan: the library atan above 2^-4; below, within 1 ulp of the correctly rounded value
    # (200-bit mpmath) and equal to it on nearly every argument
    big = fin & (np.abs(a) > 2.0 ** -4)
    assert np.array_equal(bits(o[big, 9]), bits(o[big, 10]))
    import mpmath
    mpmath.mp.prec = 200
    xs = np.concatenate([(rng.random(4000) - 0.5) * 2.0 ** -3, (rng.random(4000) - 0.5) * 2e-4,
                         (rng.random(2000) - 0.5) * 2.0 ** rng.integers(-60, -5, 2000), [0.0, -0.0, 2.0 ** -4]])
    tx = torch.from_numpy(xs).to(gpu)
    ox = torch.empty((xs.shape[0], cols), dtype=torch.float64, device=gpu)
    _lib.check(_lib.lib().akb_selftest_arith_f64(D.ptr(tx), D.ptr(tx), xs.shape[0], D.ptr(ox), D.stream_handle()))
    got = ox.cpu().numpy()[:, 9]
    cr = np.array([float(mpmath.atan(mpmath.mpf(float(x)))) for x in xs])
    ulp = np.spacing(np.abs(cr))
    assert np.all(np.abs(got - cr) <= ulp) and np.array_equal(np.signbit(got), np.signbit(cr))
    assert np.mean(got == cr) > 0.99


# ----------------------------------------------------------------------------- fused chain

def _geom():
    from akbraytracing_amd.wavefront import SystemGeometry
    return SystemGeometry.from_dict(golden_json("akb_geometry.json"))


def test_fused_chain_bitwise_vs_oracle(gpu):
    from akbraytracing_amd.trace import trace_chain
    g = _geom()
    f = golden("akb_raywave_65.npz")
    r = OPL.akb_ray_wave(golden_json("akb_geometry.json"), 65)
    th = torch.from_numpy(r["tan_h2"]).to(gpu)
    tv = torch.from_numpy(r["tan_v2"]).to(gpu)
    res = trace_chain(g.mirrors, tan_h=th, tan_v=tv, det_ghij=g.det1,
                      want=("hits", "last_hit", "dir_out", "det", "opl", "atan"))
    assert int(res.flags.item()) == 0
    assert np.array_equal(res.hits.cpu().numpy(), f["pass2_hits"])
    assert np.array_equal(res.dir_out.cpu().numpy(), r["r4"])
    assert np.array_equal(res.det.cpu().numpy(), r["det_pre"])
    segs = r["segs"]
    assert np.array_equal(res.opl.cpu().numpy(), segs[0] + segs[1] + segs[2] + segs[3])
    at = res.atan.cpu().numpy()
    assert _ulp_diff(at[0], np.arctan(r["r4"][1] / r["r4"][0])) <= 2
    assert _ulp_diff(at[1], np.arctan(r["r4"][2] / r["r4"][0])) <= 2


def test_fused_chain_explicit_dirs_and_shards(gpu):
    """explicit-direction mode and row-sharded grid launches reproduce the full-grid launch."""
    from akbraytracing_amd.trace import trace_chain
    g = _geom()
    n = 97
    rh, rv = g.angle_h.table(n), g.angle_v.table(n)
    th, tv = torch.from_numpy(np.tan(rh)).to(gpu), torch.from_numpy(np.tan(rv)).to(gpu)
    full = trace_chain(g.mirrors, tan_h=th, tan_v=tv, det_ghij=g.det1, want=("det", "opl"))
    dirs = O.normalize_vector(np.vstack([np.ones(n * n), np.tile(np.tan(rh), n), np.repeat(np.tan(rv), n)]))
    expl = trace_chain(g.mirrors, dirs=torch.from_numpy(dirs).to(gpu), det_ghij=g.det1, want=("det", "opl"))
    assert torch.equal(full.det, expl.det) and torch.equal(full.opl, expl.opl)
    parts = []
    for row0, rows in ((0, 30), (30, 40), (70, 27)):
        p = trace_chain(g.mirrors, tan_h=th, tan_v=tv, row0=row0, n_rays=rows * n, det_ghij=g.det1, want=("det",))
        parts.append(p.det)
    assert torch.equal(torch.cat(parts, dim=1), full.det)


def test_chain_flags_on_miss(gpu):
    from akbraytracing_amd.trace import Mirror, trace_chain
    sphere = Mirror([1.0, 1.0, 1.0, 0, 0, 0, 0, 0, 0, -1.0])
    dirs = torch.tensor([[1.0, 1.0], [0.0, 0.0], [0.0, 0.0]], dtype=torch.float64, device=gpu)
    src = torch.tensor([[-5.0, -5.0], [0.0, 5.0], [0.0, 0.0]], dtype=torch.float64, device=gpu)
    r = trace_chain([sphere], dirs=dirs, src=src, want=("last_hit",))
    assert int(r.flags.item()) & 0x1


# ----------------------------------------------------------------------------- sums

@pytest.mark.parametrize("n", [1, 7, 8, 100, 128, 129, 8191, 8192, 8193, 65537, 1000003])
def test_pairwise_sum_matches_numpy(gpu, n):
    from akbraytracing_amd.reduce import np_sum
    rng = np.random.default_rng(n)
    x = 146.0 + rng.standard_normal((3, n)) * 1e-3
    s, c = np_sum(torch.from_numpy(x).to(gpu))
    s = s.cpu().numpy()
    for r in range(3):
        assert s[r] == np.sum(x[r])
        assert s[r] / c[r].item() == np.mean(x, axis=1)[r]
    x[:, ::5] = np.nan
    s, c = np_sum(torch.from_numpy(x).to(gpu), nan=True)
    s, c = s.cpu().numpy(), c.cpu().numpy()
    for r in range(3):
        assert s[r] == np.nansum(x[r])
        with np.errstate(invalid="ignore"):
            assert np.array_equal(s[r] / c[r], np.nanmean(x[r]), equal_nan=True)


def test_pairwise_sum_short_buffer_sweep(gpu):
    """The last, short buffer's split tree (built level by level on the device) over many tail
    lengths, behind two full buffers and alone."""
    from akbraytracing_amd.reduce import np_sum
    rng = np.random.default_rng(11)
    tails = sorted(set([1, 2, 7, 8, 9, 15, 16, 17, 127, 128, 129, 135, 136, 255, 256, 257, 263, 264, 519, 1031,
                        2055, 4103, 4104, 8190, 8191] + list(rng.integers(1, 8192, 40))))
    for t in tails:
        for n in (int(t), 2 * 8192 + int(t)):
            x = 146.0 + rng.standard_normal((2, n)) * 1e-3
            x[1, ::7] = np.nan
            s, c = np_sum(torch.from_numpy(x).to(gpu), nan=True)
            s, c = s.cpu().numpy(), c.cpu().numpy()
            assert s[0] == np.sum(x[0]) and c[0] == n, (n, s[0] - np.sum(x[0]))
            assert s[1] == np.nansum(x[1]) and c[1] == np.count_nonzero(~np.isnan(x[1])), n


def test_tilt_params_on_device(gpu):
    """akb_tilt_params_f64: the means are numpy's divisions bit for bit and R_y, R_z hold the
    correctly rounded cos / sin (numpy's glibc values may differ by one ulp, rarely)."""
    import mpmath
    from akbraytracing_amd import _lib, device as D
    from akbraytracing_amd.primitives import rotation_matrices
    L = _lib.lib()
    rng = np.random.default_rng(3)
    mpmath.mp.prec = 200
    worst = 0
    for trial in range(64):
        cnt = rng.integers(1, 10 ** 7, 5).astype(np.int64)
        sums = (rng.standard_normal(5) * 1e-3 * cnt).astype(np.float64)
        sums[2:] = rng.standard_normal(3) * 100.0 * cnt[2:]
        s_d = torch.from_numpy(sums).to(gpu)
        c_d = torch.from_numpy(cnt).to(gpu)
        params = torch.empty(25, dtype=torch.float64, device=gpu)
        keys = torch.full((4,), 7, dtype=torch.int64, device=gpu)
        flags = torch.tensor([trial, 5, -1], dtype=torch.int32, device=gpu)
        _lib.check(L.akb_tilt_params_f64(D.ptr(s_d), D.ptr(c_d), D.ptr(params), D.ptr(keys), D.ptr(flags), 2,
                                         D.stream_handle()))
        p = params.cpu().numpy()
        assert keys.cpu().numpy().tolist() == [0, 0, 0, 0] and flags.cpu().numpy().tolist() == [0, 0, -1]
        assert params[23:25].cpu().view(torch.int32).tolist() == [trial, 5, 0, 0]  # kept before the clear
        mean = sums / cnt
        theta_y, theta_z = -mean[1], mean[0]
        assert p[0] == theta_y and p[1] == theta_z
        assert np.array_equal(p[20:23], mean[2:5])
        ry, rz = rotation_matrices(-theta_y, -theta_z)
        cy, sy = float(mpmath.cos(mpmath.mpf(-theta_y))), float(mpmath.sin(mpmath.mpf(-theta_y)))
        cz, sz = float(mpmath.cos(mpmath.mpf(-theta_z))), float(mpmath.sin(mpmath.mpf(-theta_z)))
        assert np.array_equal(p[2:11], [cy, 0, sy, 0, 1, 0, -sy, 0, cy])
        assert np.array_equal(p[11:20], [cz, -sz, 0, sz, cz, 0, 0, 0, 1])
        ulp = np.abs(np.concatenate([p[2:11] - ry.ravel(), p[11:20] - rz.ravel()])) / np.spacing(1.0)
        worst = max(worst, float(ulp.max()))
    assert worst <= 1.0


# ----------------------------------------------------------------------------- wavefront pipeline

def test_ray_wave_65_vs_reference(gpu):
    from akbraytracing_amd.wavefront import RayWave
    f = golden("akb_raywave_65.npz")
    rw = RayWave(_geom(), 65)
    out = rw.run(keep_rotated=True, full=True)
    assert out["flags"] == (0, 0)
    assert np.array_equal(out["tan_h2"].cpu().numpy(), OPL.akb_ray_wave(golden_json("akb_geometry.json"), 65)["tan_h2"])
    assert np.array_equal(out["last_hit"].cpu().numpy(), f["pass2_hits"][3])
    for key, ref in (("dir_rot", "rot_dir"), ("pt_rot", "rot_pt"), ("detcenter", "detcenter"),
                     ("detcenter2", "detcenter2"), ("dist_err2", "dist_err2"), ("wave2", "wave2")):
        got = out[key].cpu().numpy()
        print(f"{key}: bitwise={np.array_equal(got, f[ref])} ulp={_ulp_diff(got, f[ref]):.1f} "
              f"maxabs={np.max(np.abs(got - f[ref])):.3e}")
    print("theta", out["theta_y"], out["theta_z"])
    # the tilt angles come from a numpy-order mean of OCML arctans: theta may sit one ulp off
    # glibc's, which moves a rotated unit vector by ~1e-16 (a few ulp of each row's scale)
    assert _ulp_diff(out["dir_rot"].cpu().numpy(), f["rot_dir"]) <= 64
    assert _ulp_diff(out["pt_rot"].cpu().numpy(), f["rot_pt"]) <= 64
    assert _ulp_diff(out["detcenter"].cpu().numpy(), f["detcenter"]) <= 64
    assert _ulp_diff(out["detcenter2"].cpu().numpy(), f["detcenter2"]) <= 64
    assert np.max(np.abs(out["dist_err2"].cpu().numpy() - f["dist_err2"])) <= 1e-4
    assert np.max(np.abs(out["wave2"].cpu().numpy() - f["wave2"])) <= 1e-4


@pytest.mark.parametrize("n", [65, 1001])
def test_two_stream_pipeline_equals_sequential_runs(gpu, n):
    """bench.py's pipeline: each run's back half (tilt, OPD, pupil) on a second stream, beside
    the next run's pass 1 - the same bits as run() one at a time, for every run in the chain."""
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), n)
    seq = rw.run()
    want = {k: seq[k].clone() for k in ("wave2", "dist_err2", "detcenter2")}
    want_opd = rw.pupil(32)[0].clone()
    bs = torch.cuda.Stream()
    outs, opds = [], []

    def back(front):
        with torch.cuda.stream(bs):
            outs.append(rw.launch_back(front, stream=bs))
            opds.append(rw.pupil(32)[0].clone())

    fronts = [rw.launch_front()]
    for _ in range(3):
        prev = fronts[-1]
        fronts.append(rw.launch_front(overlap=lambda p=prev: back(p)))
    back(fronts[-1])
    torch.cuda.synchronize()
    assert len(outs) == 4
    for o, opd in zip(outs, opds):
        for k, v in want.items():
            assert torch.equal(o[k], v), k
        assert torch.equal(opd, want_opd)


def test_reserved_cu_stream_gives_the_same_bits(gpu):
    """bench.py's default at one GPU: the passes on a stream that leaves 40 CUs to the back stream
    (akb_stream_create_reserved) - the same bits as on torch's default stream."""
    from akbraytracing_amd.device import reserved_stream
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), 1001)
    seq = rw.run()
    want = {k: seq[k].clone() for k in ("wave2", "dist_err2", "detcenter2")}
    rs = reserved_stream(40)
    with torch.cuda.stream(rs):
        for _ in range(2):
            out = rw.run()
            for k, v in want.items():
                assert torch.equal(out[k], v), k
    torch.cuda.synchronize()


@pytest.mark.parametrize("n", [65, 1001])
def test_fused_pipeline_equals_sequential_runs(gpu, n):
    """bench.py's default pipeline: each run's tilt inside the next run's pass-1 kernel
    (akb_chain_tilt_f64), its OPD and pupil on a second stream during the next resample - the
    same bits as run() one at a time."""
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), n)
    seq = rw.run()
    want = {k: seq[k].clone() for k in ("wave2", "dist_err2", "detcenter2")}
    want_opd = rw.pupil(32)[0].clone()
    bs = torch.cuda.Stream()
    outs, opds, fused = [], [], []

    def back(front):
        fused.append(front.tilt is not None)
        with torch.cuda.stream(bs):
            outs.append(rw.launch_back(front, stream=bs))
            opds.append(rw.pupil(32)[0].clone())

    f = rw.launch_front()
    for _ in range(3):
        f = rw.launch_front(overlap=lambda p=f: back(p), fuse=f)
    back(f)
    torch.cuda.synchronize()
    assert fused == [True, True, True, False]
    for o, opd in zip(outs, opds):
        for k, v in want.items():
            assert torch.equal(o[k], v), k
        assert torch.equal(opd, want_opd)


def _fused_pipeline(rw, back, lag, kws):
    """Fronts pipelined as bench.py --fuse 2 does: run k's pass 1 tilts run k-lag and forms run
    k-lag-1's OPD (lag 2 is bench.py's: run k-1's pass-2 sums and tilt parameters then finish
    beside run k's passes); the runs left in flight drain through the tilt-only and unfused back
    halves. kws: launch_front keywords of each run. Returns the expected back-half kinds."""
    fr = []
    for kw in kws:
        if len(fr) == lag + 1:
            g = fr.pop(0)
            fr.append(rw.launch_front(overlap=lambda p=g: back(p), fuse=fr[0], fuse_opd=g, **kw))
        elif len(fr) == lag:
            fr.append(rw.launch_front(fuse=fr[0], **kw))
        else:
            fr.append(rw.launch_front(**kw))
    for f in fr:
        back(f)
    return [(True, True)] * (len(kws) - lag - 1) + [(True, False)] + [(False, False)] * lag


@pytest.mark.parametrize("lag", [1, 2])
@pytest.mark.parametrize("n", [65, 1001])
def test_opd_fused_pipeline_equals_sequential_runs(gpu, n, lag):
    """bench.py's default pipeline (--fuse 2): run k's pass-1 kernel also tilts run k-2 (or k-1)
    and forms run k-3's (k-2's) OPD maps and extent keys (akb_chain_tilt_opd_f64), the tilt sums
    finished on a stream of their own, each run's pass-2 sums and tilt parameters on another; the
    OPD-formed run's launch_back and pupil go beside pass 2 - the same bits, pupil pitch
    included, as run() one at a time."""
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), n)
    seq = rw.run()
    want = {k: seq[k].clone() for k in ("wave2", "dist_err2", "detcenter2", "total2")}
    want_opd, want_pitch = (t.clone() for t in rw.pupil(32))
    want_means = rw.means()
    bs = torch.cuda.Stream()
    outs, pupils, kinds, means = [], [], [], []

    def back(front):
        kinds.append((front.tilt is not None, front.opd is not None))
        with torch.cuda.stream(bs):
            outs.append(rw.launch_back(front, stream=bs))
            pupils.append(tuple(t.clone() for t in rw.pupil(32)))
            means.append(rw.means())

    want_kinds = _fused_pipeline(rw, back, lag, [{}] * (lag + 5))
    torch.cuda.synchronize()
    assert kinds == want_kinds
    for o, (opd, pitch), m in zip(outs, pupils, means):
        for k, v in want.items():
            assert torch.equal(o[k], v), k
        assert torch.equal(opd, want_opd) and torch.equal(pitch, want_pitch)
        for a, b in zip(m, want_means):
            assert np.array_equal(a, b)


def _variants(k):
    """k distinct systems over the reference AKB's ray grid: the last mirror's constant term and
    both detector planes moved a little per system (each run then has its own hits, tilt, means
    and OPD, so a run's tilt or OPD formed from another run's buffers cannot go unnoticed)."""
    import copy
    base = golden_json("akb_geometry.json")
    from akbraytracing_amd.wavefront import SystemGeometry
    out = []
    for i in range(k):
        d = copy.deepcopy(base)
        d["mirrors"][-1]["coeffs"][9] = d["mirrors"][-1]["coeffs"][9] * (1.0 + 2e-11 * i)
        d["det1"][9] = d["det1"][9] - 3e-6 * i
        d["det2"][9] = d["det2"][9] - 5e-6 * i
        out.append(SystemGeometry.from_dict(d))
    return out


@pytest.mark.parametrize("lag", [1, 2])
@pytest.mark.parametrize("n", [65, 301])
def test_opd_fused_pipeline_distinct_systems(gpu, n, lag):
    """The default pipeline (--fuse 2) with every run tracing another system: run k's pass-1
    kernel tilts run k-lag (with that run's detector planes and rotation) and forms run
    k-lag-1's OPD (from its tilt sums); each run's Wave2, DistError2, detector-2 hits, totals,
    means and pupil pitch equal a sequential run() of that same system, bit for bit."""
    from akbraytracing_amd.wavefront import RayWave
    systems = _variants(7)
    rw = RayWave(systems[0], n)
    want = []
    for g in systems:
        seq = rw.run(geometry=g)
        opd, pitch = rw.pupil(32)
        want.append(({k: seq[k].clone() for k in ("wave2", "dist_err2", "detcenter2", "total2")},
                     opd.clone(), pitch.clone(), rw.means()))
    # the systems really differ run to run
    assert not torch.equal(want[0][0]["wave2"], want[1][0]["wave2"])
    assert not np.array_equal(want[0][3][1], want[1][3][1])
    bs = torch.cuda.Stream()
    outs, kinds = [], []

    def back(front):
        kinds.append((front.tilt is not None, front.opd is not None))
        with torch.cuda.stream(bs):
            o = rw.launch_back(front, stream=bs)
            outs.append(({k: o[k].clone() for k in want[0][0]}, *(t.clone() for t in rw.pupil(32)), rw.means()))

    kws = [dict(geometry=g, next_geometry=systems[i + 1] if i + 1 < len(systems) else None)
           for i, g in enumerate(systems)]
    want_kinds = _fused_pipeline(rw, back, lag, kws)
    torch.cuda.synchronize()
    assert kinds == want_kinds
    for i, ((o, opd, pitch, m), (w, wopd, wpitch, wm)) in enumerate(zip(outs, want)):
        for k, v in w.items():
            assert torch.equal(o[k], v), (i, k)
        assert torch.equal(opd, wopd) and torch.equal(pitch, wpitch), i
        for a, b in zip(m, wm):
            assert np.array_equal(a, b), i


def test_prepass_for_an_unannounced_system_is_redone(gpu):
    """A run whose system differs from the one its picks prepass was queued for (no
    next_geometry) redoes the prepass: same bits as a fresh RayWave on that system."""
    from akbraytracing_amd.wavefront import RayWave
    a, b = _variants(2)
    want = RayWave(b, 65).run()["wave2"].clone()
    rw = RayWave(a, 65)
    rw.run()
    assert torch.equal(rw.run(geometry=b)["wave2"], want)
    with pytest.raises(ValueError):
        import copy
        c = copy.deepcopy(b)
        c.angle_h = type(c.angle_h)(c.angle_h.start * 1.01, c.angle_h.stop, c.angle_h.offset)
        rw.run(geometry=c)


def test_fused_pipeline_falls_back_where_it_cannot_fuse(gpu):
    """launch_front(fuse=...) on a single-detector system (KB) or a full run keeps the tilt in
    the back half and still gives run()'s bits."""
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    rw = RayWave(SystemGeometry.from_dict(golden_json("kb_geometry.json")), 65)
    want = rw.run()["dist_err"].clone()
    f = rw.launch_front()
    g = rw.launch_front(fuse=f)
    assert f.tilt is None
    assert torch.equal(rw.launch_back(f)["dist_err"], want)
    assert torch.equal(rw.launch_back(g)["dist_err"], want)
    rw = RayWave(_geom(), 65)
    want = rw.run(full=True)["sph"].clone()
    f = rw.launch_front(full=True)
    g = rw.launch_front(fuse=f)
    assert f.tilt is None
    assert torch.equal(rw.launch_back(f)["sph"], want)


def test_ray_wave_pass1_miss_raises_after_pass2(gpu):
    """A pass-1 miss outside the resample's pick rays (only the grid's corner rays miss a tiny
    sphere) is found when the flag words come back after pass 2, and the run fails as the
    reference's all-NaN rule makes it; a miss among the pick rays fails before pass 2."""
    from akbraytracing_amd import _lib
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    g = golden_json("akb_geometry.json")
    x0, radius = 1.0, 2.5e-5  # corners (|angle| ~2.8e-5) miss, the middle row / column (<2.2e-5) hit
    g = dict(g, mirrors=[{"coeffs": [1.0, 1.0, 1.0, 0.0, 0.0, 0.0, -2 * x0, 0.0, 0.0, x0 * x0 - radius ** 2],
                          "negative": True}],
             det1=[0.0] * 6 + [1.0, 0.0, 0.0, -0.5], det2=[0.0] * 6 + [1.0, 0.0, 0.0, -0.4])
    rw = RayWave(SystemGeometry.from_dict(g), 65)
    with pytest.raises(_lib.AKBError, match="pass 1"):
        rw.run()
    narrow = dict(g, mirrors=[dict(g["mirrors"][0], coeffs=g["mirrors"][0]["coeffs"][:9] + [x0 * x0 - 1e-5 ** 2])])
    with pytest.raises(_lib.AKBError, match="pass 1"):
        RayWave(SystemGeometry.from_dict(narrow), 65).run()


def test_fused_pipeline_flagged_pass2_takes_staged_path(gpu):
    """If a run's pass 2 turns out flagged after the next pass 1 already tilted it, launch_back
    discards the fused tilt and redoes the run stage by stage (here the flag is forced on a clean
    run, so the staged results must match the fused ones to the tilt stage's tolerance)."""
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), 65)
    want = rw.run()
    want = {k: want[k].clone() for k in ("wave2", "dist_err2")}
    f = rw.launch_front()
    nxt = rw.launch_front(fuse=f)
    assert f.tilt is not None
    rw._resolve(f)
    f.flags = (0, 0x1)  # as if a ray of its pass 2 had missed
    out = rw.launch_back(f)
    torch.cuda.synchronize()
    for k, v in want.items():
        assert torch.max(torch.abs(out[k] - v)).item() <= 1e-4, k
    rest = rw.launch_back(nxt)
    assert torch.equal(rest["wave2"], want["wave2"])
    # the same two runs later: a flagged run is not OPD-fused into the pass 1 after next
    f = rw.launch_front()
    nxt = rw.launch_front(fuse=f)
    rw._resolve(f)
    f.flags = (0, 0x1)
    last = rw.launch_front(fuse=nxt, fuse_opd=f)
    assert f.opd is None and nxt.tilt is not None
    out = rw.launch_back(f)
    for k, v in want.items():
        assert torch.max(torch.abs(out[k] - v)).item() <= 1e-4, k
    for fr in (nxt, last):
        assert torch.equal(rw.launch_back(fr)["wave2"], want["wave2"])


def test_config5_legendre_opl_perturbation(gpu):
    """BASELINE config 5: the chain adds the Legendre figure-error model to each ray's OPL (model
    from oracle/legendre.py; the basis is pinned to legendre_fit by test_oracle_golden)."""
    from akbraytracing_amd.legendre import LegendrePerturbation, config5_coefficients
    from akbraytracing_amd.wavefront import RayWave
    import oracle.legendre as OL
    n = 65
    for scale in (1.0, 1e6):  # the config's own size, and one far above the OPL's ulp
        c = config5_coefficients() * scale
        base = RayWave(_geom(), n).run(opd=False)
        pert = RayWave(_geom(), n, perturbation=LegendrePerturbation(c)).run(opd=False)
        want = OL.perturbation(n, n, c).reshape(-1)
        got = (pert["opl"] - base["opl"]).cpu().numpy()
        ulp = np.spacing(base["opl"].cpu().numpy())
        assert np.all(np.abs(got - want) <= 1.01 * ulp + 1e-13 * np.abs(want))
        assert torch.equal(pert["last_hit"], base["last_hit"])


@pytest.mark.parametrize("n", [65, 128, 1001])
def test_fused_means_equal_numpy_on_the_rows(gpu, n):
    """The leaf sums fused into pass 2 and the tilt kernel give the same means numpy takes of the
    rows they never write (n = 65: short last buffer only; 1001: full buffers + tail)."""
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), n)
    out = rw.run(full=True)
    at = out["atan"].cpu().numpy()
    det = out["det_pre"].cpu().numpy()
    assert out["theta_y"] == -np.nanmean(at[1]) and out["theta_z"] == np.nanmean(at[0])
    assert np.array_equal(out["focus_apprx"], np.mean(det, axis=1))
    mt, mf = rw.means()
    assert mt[0] == np.nanmean(out["total"].cpu().numpy()) and mt[1] == np.nanmean(out["total2"].cpu().numpy())
    assert np.array_equal(mf, np.nanmean(out["detcenter"].cpu().numpy(), axis=1))
    e2 = out["dist_err2"].cpu().numpy()
    assert np.array_equal(e2, (out["total2"].cpu().numpy() - mt[1]) * 1e9)


def test_kb_wave_65_vs_reference(gpu):
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    f = golden("kb_wave_65.npz")
    rw = RayWave(SystemGeometry.from_dict(golden_json("kb_geometry.json")), 65)
    out = rw.run(opd=False, full=True)
    assert np.array_equal(out["last_hit"].cpu().numpy(), f["pass2_hits"][1])
    assert np.array_equal(out["dir_out"].cpu().numpy(), f["pass2_refl"])
    assert np.array_equal(out["det_pre"].cpu().numpy(), f["pass2_det"])


# ----------------------------------------------------------------------------- PSF

def test_psf_cases(gpu):
    from akbraytracing_amd import psf as G
    d = golden("psf_cases.npz")
    for k in range(5):
        ny, nx, pad, win, eff, dy = d[f"k{k}_spec"]
        r = G.compute_psf_fft(d[f"k{k}_opd"], d[f"k{k}_amp"], 13.5e-9, 5e-6, 1e-2, pad_factor=int(pad),
                              window="hann" if win else None, return_efield=bool(eff),
                              pupil_dy_m=None if dy < 0 else dy)
        ref = d[f"k{k}_psf"]
        assert r[0].shape == ref.shape
        assert np.max(np.abs(r[0] - ref)) <= 1e-10  # peak-normalised
        assert np.array_equal(r[1], d[f"k{k}_x"]) and np.array_equal(r[2], d[f"k{k}_y"])
        if eff:
            e = d[f"k{k}_efield"]
            assert np.max(np.abs(r[3] - e)) <= 1e-10 * np.max(np.abs(e))


def test_psf_real_pupil_pad16(gpu):
    from akbraytracing_amd import psf as G
    d = golden("akb_psf_65.npz")
    I, x, y = G.compute_psf_fft(d["opd"], d["amp"], float(d["wl"]), float(d["dx"]), float(d["f"]),
                                pad_factor=int(d["pad"]), pupil_dy_m=float(d["dy"]))
    assert I.shape == tuple(d["shape"])
    y0, x0 = d["crop_origin"]
    h = d["crop"].shape[0]
    assert np.max(np.abs(I[y0:y0 + h, x0:x0 + h] - d["crop"])) <= 1e-10
    assert abs(np.sum(I) - float(d["psf_sum"])) <= 1e-9 * float(d["psf_sum"])
    assert np.array_equal(x, d["x_im"])


def test_psf_stack_equals_single(gpu):
    from akbraytracing_amd import psf as G
    d = golden("akb_psf_65.npz")
    opd = torch.from_numpy(d["opd"]).to(gpu)
    amp = torch.from_numpy(d["amp"]).to(gpu)
    lams = [13.5e-9, 1.35e-9, 1.35e-10]
    st, _, imax = G.psf_stack(opd, amp, lams, float(d["dx"]), float(d["dy"]), pad_factor=8)
    for b, lam in enumerate(lams):
        one, _, _ = G.psf_stack(opd, amp, [lam], float(d["dx"]), float(d["dy"]), pad_factor=8)
        assert torch.equal(st[b], one[0])
        ref = __import__("oracle.psf", fromlist=["psf"]).psf(d["opd"], d["amp"], lam, float(d["dx"]), 1e-2, 8,
                                                            dy=float(d["dy"]))[0]
        assert np.max(np.abs(one[0].cpu().numpy() - ref)) <= 1e-10


@pytest.mark.parametrize("ny,nx,pad,win,eff", [(128, 128, 16, False, False), (64, 32, 4, True, True),
                                               (15, 16, 3, False, True), (8, 8, 1, False, False),
                                               (256, 8, 2, True, False), (32, 256, 5, False, True),
                                               (512, 512, 8, False, True), (1024, 32, 8, True, False),
                                               (15, 16, 16, False, True), (16, 8, 8, True, True),
                                               (256, 64, 16, True, True), (64, 512, 16, False, False),
                                               (1024, 16, 16, False, True), (127, 1024, 16, True, False),
                                               (32, 1024, 16, False, True)])
def test_psf_pruned_transform(gpu, ny, nx, pad, win, eff, monkeypatch):
    """Power-of-two pupils take the pruned transform (the padded plane is never built): against
    the oracle (numpy fft2 on the padded plane), the rocFFT path on the same input and, at pad 8
    / 16 (the line transforms), the column-pass transform."""
    from akbraytracing_amd import psf as G
    import oracle.psf as OP
    rng = np.random.default_rng(ny * 7 + nx)
    opd = rng.standard_normal((ny, nx)) * 2e-9
    opd[rng.random((ny, nx)) < 0.05] = np.nan
    amp = np.where(np.isfinite(opd), 1.0, 0.0)
    lam, dx, dy = 13.5e-9, 5e-6, 4e-6
    o = torch.from_numpy(opd).to(gpu)
    fast = G.psf_stack(o, None, [lam], dx, dy, pad_factor=pad, window="hann" if win else None, return_efield=eff)
    ref = OP.psf(opd, amp, lam, dx, 1e-2, pad, "hann" if win else None, eff, dy=dy)
    got = fast[0][0].cpu().numpy()
    assert got.shape == ref[0].shape
    assert np.max(np.abs(got - ref[0])) <= 1e-10
    if eff:
        e = fast[1][0].cpu().numpy()
        assert np.max(np.abs(e - ref[3])) <= 1e-10 * np.max(np.abs(ref[3]))
    if pad in (8, 16):
        # the select route (default below 2^24 points), the row-bound rounds (default above) and
        # the fp32 peak pass only pick the rows of the exact fp64 one: identical bits on every route
        for mode in ("f64", "f32", "bound", "select"):
            monkeypatch.setenv("AKB_PSF_PEAK", mode)
            alt = G.psf_stack(o, None, [lam], dx, dy, pad_factor=pad, window="hann" if win else None,
                              workspace=G.PsfWorkspace())
            assert torch.equal(alt[0][0], fast[0][0])
        monkeypatch.delenv("AKB_PSF_PEAK")
        monkeypatch.setenv("AKB_PSF_PATH", "cols")
        cols = G.psf_stack(o, None, [lam], dx, dy, pad_factor=pad, window="hann" if win else None,
                           workspace=G.PsfWorkspace())
        assert np.max(np.abs(cols[0][0].cpu().numpy() - got)) <= 1e-12
    monkeypatch.setenv("AKB_PSF_ROCFFT", "1")
    slow = G.psf_stack(o, None, [lam], dx, dy, pad_factor=pad, window="hann" if win else None,
                       workspace=G.PsfWorkspace())
    assert np.max(np.abs(slow[0][0].cpu().numpy() - got)) <= 1e-12


def test_psf_line_1024_stack_equals_single(gpu, monkeypatch):
    """1024-point lines (two output columns a thread, 512-thread workgroups) batched over three
    wavelengths, with the E-field: each entry the single-wavelength run's bits, on every peak route."""
    from akbraytracing_amd import psf as G
    rng = np.random.default_rng(1024)
    opd = rng.standard_normal((32, 1024)) * 3e-9
    opd[rng.random((32, 1024)) < 0.03] = np.nan
    o = torch.from_numpy(opd).to(gpu)
    lams = [13.5e-9, 1.35e-9, 6.7e-9]
    base = None
    for mode in ("select", "bound", "f64", "f32"):
        monkeypatch.setenv("AKB_PSF_PEAK", mode)
        st, ef, imax = G.psf_stack(o, None, lams, 5e-6, 4e-6, pad_factor=16, return_efield=True,
                                   workspace=G.PsfWorkspace())
        if base is None:
            base = st
            for b, lam in enumerate(lams):
                one, e1, im1 = G.psf_stack(o, None, [lam], 5e-6, 4e-6, pad_factor=16, return_efield=True,
                                           workspace=G.PsfWorkspace())
                assert torch.equal(st[b], one[0]) and torch.equal(ef[b], e1[0])
                assert float(imax[b]) == float(im1[0])
        else:
            assert torch.equal(st, base), mode


@pytest.mark.parametrize("n", [128, 512])
def test_psf_line_stack_equals_single(gpu, n):
    """The line transforms batched over wavelengths (one launch per pass for the stack; at 512^2 x
    pad 16 = 8192^2 the row-bound peak route, per batch entry) equal one wavelength at a time,
    bit for bit, and the oracle at 128^2."""
    from akbraytracing_amd import psf as G
    rng = np.random.default_rng(n)
    opd = rng.standard_normal((n, n)) * 3e-9
    opd[rng.random((n, n)) < 0.03] = np.nan
    o = torch.from_numpy(opd).to(gpu)
    lams = [13.5e-9, 1.35e-9, 6.7e-9]
    st, _, imax = G.psf_stack(o, None, lams, 5e-6, 4e-6, pad_factor=16)
    for b, lam in enumerate(lams):
        one, _, im1 = G.psf_stack(o, None, [lam], 5e-6, 4e-6, pad_factor=16)
        assert torch.equal(st[b], one[0]) and torch.equal(imax[b:b + 1], im1)
        del one
    if n == 128:
        import oracle.psf as OP
        amp = np.where(np.isfinite(opd), 1.0, 0.0)
        for b, lam in enumerate(lams):
            ref = OP.psf(opd, amp, lam, 5e-6, 1e-2, 16, dy=4e-6)[0]
            assert np.max(np.abs(st[b].cpu().numpy() - ref)) <= 1e-10


@pytest.mark.parametrize("case", ["point", "zero", "nan"])
def test_psf_line_peak_edges(gpu, case, monkeypatch):
    """The line transforms' peak at its edges: one lit pixel (a flat |F|: every row ties the fp32
    peak, so the fp64 pass runs over all rows), a dark pupil (Imax = 0: the unnormalised plane) and
    an infinite amplitude (NaN in the plane: numpy's max propagates it) - against the oracle and
    against the fp64-only peak."""
    from akbraytracing_amd import psf as G
    import oracle.psf as OP
    n, pad = 64, 16
    opd = np.zeros((n, n))
    amp = np.zeros((n, n))
    if case == "point":
        amp[17, 40] = 0.75
    elif case == "nan":
        amp[:] = 1.0
        amp[5, 9] = np.inf
    o, a = torch.from_numpy(opd).to(gpu), torch.from_numpy(amp).to(gpu)
    got = G.psf_stack(o, a, [13.5e-9], 5e-6, 5e-6, pad_factor=pad)[0][0].cpu().numpy()
    with np.errstate(invalid="ignore"):
        ref = OP.psf(opd, amp, 13.5e-9, 5e-6, 1e-2, pad)[0]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = np.isfinite(ref)
    if fin.any():
        assert np.max(np.abs(got[fin] - ref[fin])) <= 1e-10 * max(1.0, np.max(np.abs(ref[fin])))
    for mode in ("f64", "f32", "bound", "select"):  # bound / select: a dark or NaN plane turns them off
        monkeypatch.setenv("AKB_PSF_PEAK", mode)
        alt = G.psf_stack(o, a, [13.5e-9], 5e-6, 5e-6, pad_factor=pad)[0][0].cpu().numpy()
        assert np.array_equal(alt, got, equal_nan=True)


@pytest.mark.parametrize("n", [128, 256])
@pytest.mark.parametrize("waves", [0.0, 0.3, 1.0, 3.0])
def test_psf_line_bound_rounds(gpu, n, waves, monkeypatch):
    """The row-bound peak (akb_psf.hip k_psf_rowbound) and the select route (pass-1 row sums and
    centre samples): from a flat wavefront (the peak row alone in round 1) to three waves of
    aberration (peak / max bound ~0.28, so round 2 runs rows under round 1's threshold) - the same
    bits as the fp64 pass over every row, and the oracle."""
    from akbraytracing_amd import psf as G
    import oracle.psf as OP
    lam = 13.5e-9
    y, x = np.mgrid[-1:1:n * 1j, -1:1:n * 1j]
    r2 = x * x + y * y
    ph = waves * (0.7 * (2 * r2 - 1) + 1.5 * x * y + 0.4 * (3 * r2 - 2) * x + 0.3 * np.sin(7 * x + 3 * y))
    opd = np.where(r2 <= 1.0, ph * lam, np.nan)
    o = torch.from_numpy(opd).to(gpu)
    monkeypatch.setenv("AKB_PSF_PEAK", "bound")  # the default from 4096^2 up
    got, _, imax = G.psf_stack(o, None, [lam], 5e-6, 5e-6, pad_factor=16)
    monkeypatch.setenv("AKB_PSF_PEAK", "f64")
    alt, _, imax64 = G.psf_stack(o, None, [lam], 5e-6, 5e-6, pad_factor=16, workspace=G.PsfWorkspace())
    assert torch.equal(alt, got) and torch.equal(imax, imax64)
    # the select route (the default below 2^24 points): the rows whose bound reaches the centre
    # samples' lower bound - few when focused, more as the aberration moves the peak off centre
    monkeypatch.setenv("AKB_PSF_PEAK", "select")
    sel, _, imaxs = G.psf_stack(o, None, [lam], 5e-6, 5e-6, pad_factor=16, workspace=G.PsfWorkspace())
    assert torch.equal(sel, got) and torch.equal(imaxs, imax64)
    if n == 128:
        amp = np.where(np.isfinite(opd), 1.0, 0.0)
        ref = OP.psf(opd, amp, lam, 5e-6, 1e-2, 16)[0]
        assert np.max(np.abs(got[0].cpu().numpy() - ref)) <= 1e-10


def test_psf_errors(gpu):
    from akbraytracing_amd import psf as G
    with pytest.raises(ValueError):
        G.compute_psf_fft(np.zeros((4, 4)), np.zeros((4, 5)), 1e-9, 1e-6, 1e-2)
    with pytest.raises(ValueError):
        G.compute_psf_fft(np.zeros((4, 4)), np.zeros((4, 4)), 1e-9, 1e-6, 1e-2, pad_factor=1.5)
    with pytest.raises(ValueError):
        G.compute_psf_fft(np.zeros((4, 4)), np.zeros((4, 4)), 1e-9, 1e-6, 1e-2, window="tukey")


# ----------------------------------------------------------------------------- focus sweeps

def test_find_defocus_vs_reference(gpu):
    """find_defocus on the reference's own 65x65 pass-2 rays: the first loop's np.std sizes on
    all 50 planes bit for bit, and the search's answer exactly."""
    from akbraytracing_amd import focus as F
    f = golden("akb_focus_65.npz")
    s2f = float(f["s2f_middle"])
    sw = F.PlaneSweep(f["reflect4"], f["points"])
    a = np.linspace(-0.3, 0.3, 50)
    size_h, size_v = sw.std(np.array([-(s2f + a[i]) for i in range(50)]))
    assert np.array_equal(size_h, f["size_h0"]) and np.array_equal(size_v, f["size_v0"])
    assert F.find_defocus(f["reflect4"], f["points"], s2f, 0.0, 65, sweep=sw) == f["best_a"]


def test_plane_sweep_subset_vs_oracle(gpu):
    """compare_sep-style thinned subsets (every ray_num-th ray, :9277-9280) against the oracle's
    plane intersection + np.std."""
    from akbraytracing_amd import focus as F
    f = golden("akb_focus_65.npz")
    sub = np.arange(4225)[32::65]
    j = -(float(f["s2f_middle"]) + np.linspace(-0.01, 0.01, 7))
    sh, sv = F.plane_std_sweep(f["reflect4"], f["points"], j, subset=sub)
    for p in range(7):
        det = O.plane_ray_intersection([0] * 6 + [1.0, 0.0, 0.0, j[p]], f["reflect4"][:, sub], f["points"][:, sub])
        assert sh[p] == np.std(det[1]) and sv[p] == np.std(det[2])


@pytest.mark.parametrize("m", [1000, 8192, 100003])
def test_plane_sweep_fused_equals_rows_and_numpy(gpu, m):
    """The fused sweep (leaf sums, no rows) gives the row variant's and numpy's np.std bits, on
    short, one-buffer and many-buffer + tail ray counts."""
    from akbraytracing_amd import focus as F
    rng = np.random.default_rng(m)
    d = np.vstack([np.ones(m), 1e-3 * rng.standard_normal(m), 1e-3 * rng.standard_normal(m)])
    d /= np.linalg.norm(d, axis=0)
    p = np.vstack([145.0 + rng.random(m), 1e-4 * rng.standard_normal(m), 1e-4 * rng.standard_normal(m)])
    j = -(146.0 + np.linspace(-0.3, 0.3, 9))
    fused = F.PlaneSweep(d, p).std(j)
    rows = F.PlaneSweep(d, p, fused=False).std(j)
    assert np.array_equal(fused[0], rows[0]) and np.array_equal(fused[1], rows[1])
    for k in (0, 4, 8):
        det = O.plane_ray_intersection([0] * 6 + [1.0, 0.0, 0.0, j[k]], d, p)
        assert fused[0][k] == np.std(det[1]) and fused[1][k] == np.std(det[2])


# ----------------------------------------------------------------------------- wave data (f3)

def test_calc_ds_vs_reference(gpu):
    from akbraytracing_amd import wavedata as W
    f = golden("akb_raywave_65.npz")
    d = golden("wavedata_65.npz")
    for k in range(4):
        assert np.array_equal(W.calc_dS(f["pass2_hits"][k], 65, 65), d["ds"][k])


def test_wave_data_files_and_chain(gpu, tmp_path):
    """saveWaveData's file set from a traced system, read back the way the Wavecalc driver reads
    it, and that driver's source -> M1..M4 -> image chain on the device against the oracle's
    Huygens sums (17 x 17 grids: every 4th ray of the 65 x 65 run)."""
    from akbraytracing_amd import wavedata as W
    f = golden("akb_raywave_65.npz")
    hits = f["pass2_hits"].reshape(4, 3, 65, 65)[:, :, ::4, ::4].reshape(4, 3, -1)
    det = f["detcenter"].reshape(3, 65, 65)[:, ::4, ::4].reshape(3, -1)
    det2 = f["detcenter2"].reshape(3, 65, 65)[:, ::4, ::4].reshape(3, -1)
    W.save_wave_data(str(tmp_path), np.zeros((3, 1)), list(hits), 17, 17, det, det2, defocus_for_wave=1e-2)
    names = sorted(p.name for p in tmp_path.iterdir())
    assert names == ["calculation_conditions.txt", "points_M1.npy", "points_M2.npy", "points_M3.npy",
                     "points_M4.npy", "points_gridDefocus.npy", "points_gridImage.npy", "points_source.npy"]
    m1 = np.load(tmp_path / "points_M1.npy")
    assert m1.shape == (4, 289) and np.array_equal(m1[3], O.calc_dS(hits[0], 17, 17).ravel())
    c = W.read_conditions(str(tmp_path))
    assert c["pix_y"] == 17 and c["ray_num_V2"] == 17 and c["option_AKB"] and c["option_HighNA"]
    out = tmp_path / "fields"
    fields = W.run_wave_chain(str(tmp_path), str(out))
    assert sorted(fields) == ["Image", "Image2", "M1", "M2", "M3", "M4"]
    # the same chain with the oracle's Huygens sums
    k = 2 * np.pi / 13.5e-9
    prev = (np.zeros((3, 1)), np.ones(1, dtype=complex), np.ones(1))
    for i in range(4):
        pts = np.load(tmp_path / f"points_M{i + 1}.npy")
        u = O.huygens_c(pts[0], pts[1], pts[2], prev[0][0], prev[0][1], prev[0][2], prev[1] * prev[2], k)
        assert np.max(np.abs(fields[f"M{i + 1}"] - u)) <= 1e-9 * np.max(np.abs(u)), i
        assert np.array_equal(np.load(out / f"complex_data_M{i + 1}.npz")["data"], fields[f"M{i + 1}"])
        prev = (pts[:3], fields[f"M{i + 1}"], pts[3])


# ----------------------------------------------------------------------------- psf_calc

def test_rotate_with_nan_vs_oracle(gpu):
    from akbraytracing_amd import psfcalc as G
    import oracle.psfcalc as PC
    d = golden("scipy_rotate.npz")
    for k in range(4):
        img = d[f"k{k}_in"].copy()
        img[d[f"k{k}_mask"] == 0] = np.nan
        ang = float(d[f"k{k}_angle"])
        got, opd = G.rotate_with_nan(torch.from_numpy(img).to(gpu), ang)
        want = PC.rotate_with_nan(img, ang)
        got = got.cpu().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(want))
        assert np.nanmax(np.abs(got - want)) <= 1e-12 * max(1.0, np.nanmax(np.abs(want)))
        assert np.array_equal(opd.cpu().numpy(), got * 1e-9, equal_nan=True)


def test_psf_calc_vs_reference(gpu, tmp_path):
    """The reference's psf_calc inputs from its 65x65 ray_wave run -> rotation, rotated pupil,
    trimmed PSF and the saved .npy files."""
    from akbraytracing_amd import psfcalc as G
    f = golden("akb_psfcalc_65.npz")
    r = G.psf_calc(f["psf_calc_in"], f["grid_H"], f["grid_V"], float(f["defocus"]), directory=str(tmp_path))
    assert r["rot"] == f["rot"]
    rot = r["rotated"].cpu().numpy()
    assert np.array_equal(np.isnan(rot), np.isnan(f["rotated"]))
    assert np.nanmax(np.abs(rot - f["rotated"])) <= 1e-12
    t = r["psf_trimmed"].cpu().numpy()
    assert t.shape == f["psf_trimmed"].shape
    assert np.max(np.abs(t - f["psf_trimmed"])) <= 1e-10
    assert np.array_equal(r["x_trimmed"], f["x_im"][f["trim_ix"]])
    assert np.array_equal(np.load(tmp_path / "psf_x.npy"), f["x_im"])
    assert np.load(tmp_path / "psf.npy").shape == (1056, 1056)


# ----------------------------------------------------------------------------- pupil map

def test_plane_correction_vs_reference(gpu):
    """plane_correction_with_nan_and_outlier_filter on the reference's 65x65 ray_wave map:
    1e-12 of the map's range (curve_fit's own tolerance; observed ~4e-14 nm on 0.23 nm)."""
    from akbraytracing_amd import pupilmap as PM
    f = golden("akb_psfcalc_65.npz")
    got = PM.plane_correction_with_nan_and_outlier_filter(f["plane_in"])
    want = f["plane_out"]
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.nanmax(np.abs(got - want)) <= 1e-12 * (np.nanmax(want) - np.nanmin(want))


@pytest.mark.parametrize("ny,nx", [(65, 65), (40, 97), (513, 511)])
def test_plane_correction_vs_oracle(gpu, ny, nx):
    """NaN border, a tilted quadratic, noise and injected outliers that the 3-sigma filter drops."""
    from akbraytracing_amd import pupilmap as PM
    import oracle.pupilmap as OPM
    rng = np.random.default_rng(ny * 1000 + nx)
    y, x = np.mgrid[0:ny, 0:nx].astype(np.float64)
    m = 0.3 + 0.02 * x - 0.01 * y + 1e-4 * x * x + 3e-5 * y * y + 0.01 * rng.standard_normal((ny, nx))
    m[((x - nx / 2) / (nx / 2)) ** 2 + ((y - ny / 2) / (ny / 2)) ** 2 > 0.9] = np.nan
    idx = rng.choice(ny * nx, size=max(3, ny * nx // 200), replace=False)
    m.flat[idx] += 0.5 * rng.choice([-1, 1], size=idx.size)
    want = OPM.plane_correction_with_nan_and_outlier_filter(m)
    got = PM.plane_correction_with_nan_and_outlier_filter(m)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.nanmax(np.abs(got - want)) <= 1e-11 * (np.nanmax(want) - np.nanmin(want))
    t = PM.plane_correction_with_nan_and_outlier_filter(torch.from_numpy(m).to(gpu))
    assert t.is_cuda and np.array_equal(t.cpu().numpy(), got, equal_nan=True)


def test_plane_correction_too_few_points(gpu):
    from akbraytracing_amd import pupilmap as PM
    m = np.full((8, 8), np.nan)
    m[0, :3] = 1.0
    with pytest.raises(TypeError):
        PM.plane_correction_with_nan_and_outlier_filter(m)


def test_match_legendre_multi_vs_reference(gpu):
    """legendre_fit.match_legendre_multi on the 65x65 wave map: inner products and fits bit for
    bit (numpy-order nansums on the device, scipy's Legendre values)."""
    from akbraytracing_amd import pupilmap as PM
    d = golden("legendre_cases.npz")
    fits, coefs, orders = PM.match_legendre_multi(d["wave_map"], 5)
    assert orders == [tuple(o) for o in d["orders"]]
    assert np.array_equal(coefs, d["coefs"])
    assert np.array_equal(fits, d["fit"])


def test_match_legendre_multi_nan_and_nonsquare(gpu):
    from akbraytracing_amd import pupilmap as PM
    rng = np.random.default_rng(5)
    m = rng.standard_normal((62, 62))
    m[:3, :] = np.nan
    m[10:20, 40:50] = np.nan
    got_f, got_c, _ = PM.match_legendre_multi(m, 4)
    from scipy.special import legendre
    xs = np.linspace(-1, 1, 62)
    for k, (ny, nx) in enumerate(PM.legendre_orders(4)):
        Z = np.outer(legendre(ny)(xs), legendre(nx)(xs))
        Z /= np.sqrt(np.nansum(Z * Z))
        c = np.nansum(Z * m)
        assert got_c[k] == c
        assert np.array_equal(got_f[k], c * Z)
    with pytest.raises(ValueError):
        PM.match_legendre_multi(np.zeros((4, 5)), 3)


# ----------------------------------------------------------------------------- griddata (f1)

def _scale_tol(ref):
    """1e-6 of the map's range, or 64 ulp of its largest magnitude (the 65x65 Wave2 carries a
    ~1e7 nm offset, so rounding alone is ~1e-8 there)."""
    return max(1e-6 * (np.nanmax(ref) - np.nanmin(ref)), 64 * np.spacing(np.nanmax(np.abs(ref))))


def test_griddata_cubic_vs_reference(gpu):
    """The driver's griddata(cubic) of Wave2 on its 65x65 detector hits (the reference's output):
    same NaN mask (outside the hull), values to rounding."""
    from akbraytracing_amd.griddata import griddata
    f = golden("akb_raywave_65.npz")
    g = golden("akb_psfcalc_65.npz")
    d2 = f["detcenter2"]
    got = griddata((d2[1, :], d2[2, :]), f["wave2"], (g["grid_H0"], g["grid_V0"]), method="cubic")
    ref = g["griddata_wave2"]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.nanmax(np.abs(got - ref)) <= _scale_tol(ref)


def _lattice(nv, nh, seed):
    u, v = np.meshgrid(np.linspace(-1, 1, nh), np.linspace(-1, 1, nv))
    X = u * 1e-4 + 3e-6 * v ** 2 - 2e-6 * u * v + 1e-6 * v ** 3
    Y = v * 1.3e-4 + 4e-6 * u ** 2 + 1e-6 * u ** 3
    rng = np.random.default_rng(seed)
    F = 0.3 * u ** 2 - 0.2 * u * v + 0.1 * np.sin(3 * v) + 1e-3 * rng.standard_normal(u.shape)
    return X, Y, F


@pytest.mark.parametrize("nv,nh", [(97, 113), (280, 300)])
def test_griddata_cubic_vs_scipy(gpu, nv, nh):
    """Deformed lattices with concave and convex edges vs scipy.interpolate.griddata itself."""
    from scipy.interpolate import griddata as sp_griddata
    from akbraytracing_amd.griddata import griddata
    X, Y, F = _lattice(nv, nh, nv)
    gx = np.linspace(X.min(), X.max(), nh)
    gy = np.linspace(Y.min(), Y.max(), nv)
    GH, GV = np.meshgrid(gx, gy)
    want = sp_griddata((X.ravel(), Y.ravel()), F.ravel(), (GH, GV), method="cubic")
    got = griddata((X.ravel(), Y.ravel()), F.ravel(), (GH, GV), method="cubic")
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.nanmax(np.abs(got - want)) <= _scale_tol(want)


@pytest.mark.parametrize("nv,nh,m", [(97, 113, 40), (280, 300, 128), (300, 280, 7), (33, 257, 300)])
def test_griddata_cell_claim_equals_triangle_claim(gpu, monkeypatch, nv, nh, m):
    """The per-cell claim kernel (index boxes estimated from the linspace axes) claims exactly the
    targets the per-triangle kernel does: the same values and NaN mask, bit for bit."""
    from akbraytracing_amd.griddata import CubicGrid
    X, Y, F = _lattice(nv, nh, nv * 7 + nh)
    X = X * (nh / nv)  # square-ish cells for the wide grids (a triangulable lattice)
    gx = np.linspace(X.min(), X.max(), m)
    gy = np.linspace(Y.min() - 1e-6, Y.max(), m + 3)  # some targets outside the hull
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    got = cg.interp(F.ravel(), gx, gy).cpu().numpy()
    monkeypatch.setenv("AKB_GD_CLAIM_TRI", "1")
    want = cg.interp(F.ravel(), gx, gy).cpu().numpy()
    assert np.array_equal(got, want, equal_nan=True)


@pytest.mark.parametrize("nv,nh,m,kind", [(97, 113, 40, "linspace"), (280, 300, 128, "linspace"),
                                          (300, 280, 7, "linspace"), (33, 257, 300, "linspace"),
                                          (97, 113, 60, "geometric"), (97, 113, 60, "repeated")])
def test_griddata_fused_cell_claims(gpu, nv, nh, m, kind):
    """The cell pass with the claims fused in (akb_gd_cells_claims_f64, then the pockets'
    akb_gd_claim_pockets_f64 - FaithfulPupil's split) gives the two-pass claims' owners
    (akb_gd_claims_f64) bit for bit, and akb_gd_cells_f64's diagonals and flags."""
    import torch
    from akbraytracing_amd import _lib
    from akbraytracing_amd import device as D
    from akbraytracing_amd.griddata import CubicGrid
    L = _lib.lib()
    X, Y, F = _lattice(nv, nh, nv * 5 + nh)
    X = X * (nh / nv)
    lo, hi = X.min(), X.max()
    if kind == "linspace":
        gx = np.linspace(lo, hi, m)
    elif kind == "geometric":
        gx = lo + (hi - lo) * (np.geomspace(1, 50, m) - 1) / 49
    else:
        gx = np.repeat(np.linspace(lo, hi, m // 2), 2)
    gy = np.linspace(Y.min() - 1e-6, Y.max(), m + 3)
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    dev = cg.x.device
    tgx, tgy = torch.tensor(gx, device=dev), torch.tensor(gy, device=dev)
    mx, my = gx.size, gy.size
    want = torch.empty(mx * my, dtype=torch.int32, device=dev)
    _lib.check(L.akb_gd_claims_f64(D.ptr(cg.x), D.ptr(cg.y), nv, nh, D.ptr(cg.diag), cg.npock, D.ptr(cg.ptri),
                                   D.ptr(cg.pnbr), D.ptr(cg.edge_tri), 0, -1, 1, D.ptr(tgx), mx, D.ptr(tgy), my,
                                   D.ptr(want), None, None))
    got = torch.empty_like(want)
    diag = torch.empty_like(cg.diag)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(L.akb_gd_cells_claims_f64(D.ptr(cg.x), D.ptr(cg.y), nv, nh, D.ptr(diag), 1e-10, D.ptr(flags),
                                         D.ptr(tgx), mx, D.ptr(tgy), my, D.ptr(got), None))
    _lib.check(L.akb_gd_claim_pockets_f64(D.ptr(cg.x), D.ptr(cg.y), nv, nh, D.ptr(diag), cg.npock, D.ptr(cg.ptri),
                                          D.ptr(tgx), mx, D.ptr(tgy), my, D.ptr(got), None))
    torch.cuda.synchronize()
    assert torch.equal(diag, cg.diag)
    flags2 = torch.zeros(1, dtype=torch.int32, device=dev)
    ring = torch.empty(2 * cg.L, dtype=torch.float64, device=dev)
    _lib.check(L.akb_gd_cells_f64(D.ptr(cg.x), D.ptr(cg.y), nv, nh, D.ptr(diag), 1e-10, D.ptr(flags2),
                                  D.ptr(ring[:cg.L]), D.ptr(ring[cg.L:]), None))
    torch.cuda.synchronize()
    assert int(flags.item()) == int(flags2.item())
    assert torch.equal(got, want)
    claimed = (want != np.iinfo(np.int32).max).float().mean().item()
    assert 0.3 < claimed < 1.0  # targets inside and outside the hull


@pytest.mark.parametrize("kind", ["geometric", "jittered", "repeated"])
def test_griddata_nonuniform_axes(gpu, monkeypatch, kind):
    """Target axes that are ascending but not evenly spaced take the binary-search claim inside the
    per-cell kernel: the same claims as the per-triangle kernel, and scipy's values."""
    from scipy.interpolate import griddata as sp_griddata
    from akbraytracing_amd.griddata import CubicGrid, griddata
    nv, nh = 97, 113
    X, Y, F = _lattice(nv, nh, 11)
    lo, hi = X.min(), X.max()
    if kind == "geometric":
        gx = lo + (hi - lo) * (np.geomspace(1, 50, 60) - 1) / 49
    elif kind == "jittered":
        gx = np.sort(np.linspace(lo, hi, 60) + np.random.default_rng(3).uniform(-0.3, 0.3, 60) * (hi - lo) / 59)
    else:
        gx = np.repeat(np.linspace(lo, hi, 30), 2)
    gy = np.linspace(Y.min(), Y.max(), 45)
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    got = cg.interp(F.ravel(), gx, gy).cpu().numpy()[0]
    monkeypatch.setenv("AKB_GD_CLAIM_TRI", "1")
    assert np.array_equal(got, cg.interp(F.ravel(), gx, gy).cpu().numpy()[0], equal_nan=True)
    monkeypatch.delenv("AKB_GD_CLAIM_TRI")
    GH, GV = np.meshgrid(gx, gy)
    want = sp_griddata((X.ravel(), Y.ravel()), F.ravel(), (GH, GV), method="cubic")
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.isfinite(got).mean() > 0.8
    assert np.nanmax(np.abs(got - want)) <= _scale_tol(want)
    assert np.array_equal(griddata((X.ravel(), Y.ravel()), F.ravel(), (GH, GV), grid_shape=(nv, nh)), got, equal_nan=True)


def test_griddata_default_tol_margin(gpu):
    """At the default stopping tolerance (scipy's 1e-6) the gridded values sit within 1e-6 of the range
    of scipy's on a coarse grid (the 65x65 reference run), and - on that grid and on a strongly
    distorted lattice - within a tenth of that bar of a 1e-12 solve: the stopping point leaves the
    parity bar its margin. (On the distorted lattice scipy itself is not the reference: qhull
    triangulates its wide boundary pockets by its own roundoff, as in near-cocircular cells.)"""
    from akbraytracing_amd.griddata import GRADIENT_TOL, CubicGrid
    assert GRADIENT_TOL <= 1e-6
    f = golden("akb_raywave_65.npz")
    g = golden("akb_psfcalc_65.npz")
    d2 = f["detcenter2"]
    cases = [(d2[1], d2[2], f["wave2"], 65, 65, g["grid_H0"][0], g["grid_V0"][:, 0], g["griddata_wave2"])]
    nv, nh = 61, 67
    u, v = np.meshgrid(np.linspace(-1, 1, nh), np.linspace(-1, 1, nv))
    X = u * 1e-4 + 2.5e-5 * v ** 2 - 1.5e-5 * u * v
    Y = v * 1.1e-4 + 2e-5 * u ** 2 + 1e-5 * u ** 3
    F = np.sin(2.5 * u) * np.cos(1.7 * v) + 0.4 * u * v
    cases.append((X.ravel(), Y.ravel(), F.ravel(), nv, nh, np.linspace(X.min(), X.max(), 50),
                  np.linspace(Y.min(), Y.max(), 50), None))
    for i, (x, y, val, a, b, ax, ay, ref) in enumerate(cases):
        cg = CubicGrid(x, y, a, b)
        got = cg.interp(val, ax, ay).cpu().numpy()[0]
        sweeps = cg.sweeps
        tight = cg.interp(val, ax, ay, tol=1e-12).cpu().numpy()[0]
        rng_ = np.nanmax(tight) - np.nanmin(tight)
        if ref is not None:
            assert np.array_equal(np.isnan(got), np.isnan(ref)), i
            assert np.nanmax(np.abs(got - ref)) <= _scale_tol(ref), i
        d = np.nanmax(np.abs(got - tight))
        print(f"case {i}: {sweeps} sweeps to the default tolerance, {d / rng_:.2e} of the range from a 1e-12 solve")
        assert d <= 0.1 * max(1e-6 * rng_, 64 * np.spacing(np.nanmax(np.abs(tight)))), i


def test_griddata_flagged_triangulation_stays_refused(gpu):
    """A triangulation the pocket check flags is refused on the first gradient call and on every later
    one (the failing status is kept, not only the fact that it was read) - by interp and by the
    cone solve, whichever comes first."""
    from akbraytracing_amd import _lib
    from akbraytracing_amd.griddata import CubicGrid
    X, Y, F = _lattice(40, 50, 2)
    cg = CubicGrid(X.ravel(), Y.ravel(), 40, 50)
    cg._status.fill_(2)  # as k_gd_check_pockets raises bit 1 (an edge that is not locally Delaunay)
    gx, gy = np.linspace(X.min(), X.max(), 9), np.linspace(Y.min(), Y.max(), 7)
    for _ in range(3):
        with pytest.raises(_lib.AKBError):
            cg.interp(F.ravel(), gx, gy)
        with pytest.raises(_lib.AKBError):
            cg.interp_cone(F.ravel(), gx, gy)
    cg2 = CubicGrid(X.ravel(), Y.ravel(), 40, 50)
    cg2._status.fill_(2)
    for _ in range(2):  # the cone solve first: refused on the first call and again on the second
        with pytest.raises(_lib.AKBError):
            cg2.interp_cone(F.ravel(), gx, gy)


def _interp_k_sweeps(cg, vals, gx, gy, K):
    """akb_gd_eval_f64 on the global Chebyshev iteration's gradients after exactly K sweeps."""
    from akbraytracing_amd import _lib
    from akbraytracing_amd import device as D
    f = vals if isinstance(vals, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(vals))
    f = f.to(cg.dev).reshape(-1, cg.nv * cg.nh).contiguous()
    grad = cg.gradients(f, maxiter=K, check_every=K, adaptive=False, tol=0.0)
    gxt, gyt = torch.from_numpy(gx).to(cg.dev), torch.from_numpy(gy).to(cg.dev)
    mx, my, nv = gx.size, gy.size, int(f.shape[0])
    owner = torch.empty(mx * my, dtype=torch.int32, device=cg.dev)
    out = torch.empty((nv, my, mx), dtype=torch.float64, device=cg.dev)
    _lib.check(_lib.lib().akb_gd_eval_f64(*cg._tri_args(), D.ptr(gxt), mx, D.ptr(gyt), my, D.ptr(f), D.ptr(grad), nv,
                                          D.ptr(owner), D.ptr(out), D.stream_handle()))
    return out.cpu().numpy()


@pytest.mark.parametrize("nv,nh,m,nvals", [(97, 113, 40, 1), (280, 300, 128, 2), (300, 280, 57, 1), (70, 530, 90, 3)])
def test_gradient_cone_equals_global_sweeps(gpu, nv, nh, m, nvals):
    """The cone solve (a patch per interior target cell, the boundary band with its pocket chords
    globally) gives the global iteration's K-sweep values bit for bit at every target, for K from 1
    to the maximum, one to three value sets, targets inside the lattice, in its pockets and outside."""
    from akbraytracing_amd.griddata import CubicGrid
    X, Y, F = _lattice(nv, nh, nv + 3 * nh)
    X = X * (nh / nv)
    vals = np.stack([F.ravel(), np.cos(3 * F.ravel()), F.ravel() ** 2])[:nvals]
    gx = np.linspace(X.min(), X.max(), m)
    gy = np.linspace(Y.min() - 1e-6, Y.max(), m + 5)
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    for K in (1, 2, 3, 7, 12, 14):
        got = cg.interp_cone(vals, gx, gy, sweeps=K).cpu().numpy()
        want = _interp_k_sweeps(cg, vals, gx, gy, K)
        assert np.array_equal(got, want, equal_nan=True), K
    assert np.isfinite(got).mean() > 0.5
    assert int(cg.cone_change[0].item()) >= 0 and int(cg.cone_change[1].item()) >= 0


def test_gradient_cone_on_the_c3_hits(gpu):
    """The cone solve on the C3 trace's own 1001^2 hits onto the 128^2 pupil: bit for bit the global
    CONE_SWEEPS-sweep values, and within 3e-7 of the range of the fully converged (1e-13) map
    (measured 1.7e-7 at 12 sweeps, 1.2e-8 at 14)."""
    from akbraytracing_amd.griddata import CONE_SWEEPS, CubicGrid
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    n = 1001
    out = RayWave(SystemGeometry.from_dict(golden_json("akb_geometry.json")), n).run()
    y, z = out["detcenter2"][1].contiguous(), out["detcenter2"][2].contiguous()
    w2 = out["wave2"].reshape(1, -1).contiguous()
    cg = CubicGrid(y, z, n, n)
    ext = cg.extent
    gx, gy = np.linspace(ext[0], ext[1], 128), np.linspace(ext[2], ext[3], 128)
    got = cg.interp_cone(w2, gx, gy).cpu().numpy()[0]
    assert np.array_equal(got, _interp_k_sweeps(cg, w2, gx, gy, CONE_SWEEPS)[0], equal_nan=True)
    ref = cg.interp(w2, gx, gy, tol=1e-13).cpu().numpy()[0]
    rng_ = np.nanmax(ref) - np.nanmin(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    err = np.nanmax(np.abs(got - ref)) / rng_
    print(f"cone ({CONE_SWEEPS} sweeps) vs converged: {err:.2e} of the range; change at the corners "
          f"{cg.cone_change.cpu().numpy().view(np.float64)[0]:.2e}, value-error estimate "
          f"{cg.cone_change.cpu().numpy().view(np.float64)[1] / rng_:.2e} of the range")
    assert err <= 3e-7


@pytest.mark.parametrize("case", ["65", "1001", "3163"])
def test_pupil_post_equals_host_chain(gpu, case):
    """akb_pupil_post_f64 (one launch: nanmean removal, plane correction, rotation estimate,
    rotate_with_nan) against the host-driven chain (pupilmap's moments + numpy solves, psfcalc's
    rotation), on the reference's 65^2 gridded map and on its 1001^2 / 3163^2 128^2 maps."""
    from akbraytracing_amd import pupilmap as PM
    from akbraytracing_amd import psfcalc as PC
    if case == "65":
        m = golden("akb_psfcalc_65.npz")["plane_in"]
    else:
        m = golden("akb_raywave_full.npz")[f"n{case}_map_wave"]
    m = m + 7.0  # a nanmean to remove
    md = torch.from_numpy(m).cuda()
    o = PM.pupil_post(md)
    PM.pupil_post_check(o["params"])
    p = o["params"].cpu().numpy()
    assert p[1] == np.isfinite(m).sum()
    assert p[0] == np.nanmean(m)  # numpy's own pairwise order
    z = md - float(np.nanmean(m))
    want = PM.plane_correction_with_nan_and_outlier_filter(z)
    got = o["corrected"]
    rng_ = float(np.nanmax(want.cpu().numpy()) - np.nanmin(want.cpu().numpy()))
    assert torch.equal(torch.isnan(got), torch.isnan(want))
    assert float(torch.nan_to_num(got - want).abs().max()) <= 1e-12 * rng_
    rot = PC.rotation_estimate(want)
    assert abs(p[11] - rot) <= 2 * np.spacing(abs(rot)) if rot == rot else p[11] != p[11]
    rw, opd = PC.rotate_with_nan(want, np.degrees(rot))
    assert torch.equal(torch.isnan(o["rotated"]), torch.isnan(rw))
    assert float(torch.nan_to_num(o["rotated"] - rw).abs().max()) <= 1e-12 * rng_
    assert torch.equal(torch.isnan(o["opd"]), torch.isnan(opd))


def test_gd_axes_equal_numpy_linspace(gpu):
    """akb_gd_axes_f64: np.linspace(min, max, m) of the ring's coordinates, bit for bit."""
    from akbraytracing_amd import _lib
    from akbraytracing_amd import device as D
    rng = np.random.default_rng(4)
    for L, mx, my in ((12648, 128, 128), (4000, 65, 1001), (7, 2, 3), (100, 1, 5)):
        rx, ry = rng.standard_normal(L) * 1e-3 + 0.02, rng.standard_normal(L) * 2e-3 - 0.01
        drx, dry = torch.from_numpy(rx).cuda(), torch.from_numpy(ry).cuda()
        gx, gy = torch.empty(mx, dtype=torch.float64).cuda(), torch.empty(my, dtype=torch.float64).cuda()
        ext = torch.empty(6, dtype=torch.float64).cuda()
        _lib.check(_lib.lib().akb_gd_axes_f64(D.ptr(drx), D.ptr(dry), L, mx, my, D.ptr(gx), D.ptr(gy), D.ptr(ext),
                                               D.stream_handle()))
        assert np.array_equal(gx.cpu().numpy(), np.linspace(rx.min(), rx.max(), mx))
        assert np.array_equal(gy.cpu().numpy(), np.linspace(ry.min(), ry.max(), my))
        assert np.array_equal(ext.cpu().numpy()[:4], [rx.min(), rx.max(), ry.min(), ry.max()])
        # the pitch psf_calc takes once the driver has subtracted the meshgrids' means (:3698, :1176)
        gh, gv = np.meshgrid(gx.cpu().numpy(), gy.cpu().numpy())
        gh, gv = gh - np.mean(gh), gv - np.mean(gv)
        if mx > 1:
            assert ext[4].item() == np.abs(gh[0, 1] - gh[0, 0])
        if my > 1:
            assert ext[5].item() == np.abs(gv[1, 0] - gv[0, 0])


def test_griddata_batched_values_and_errors(gpu):
    from akbraytracing_amd import _lib
    from akbraytracing_amd.griddata import CubicGrid, griddata
    X, Y, F = _lattice(40, 50, 1)
    gx = np.linspace(X.min(), X.max(), 50)
    gy = np.linspace(Y.min(), Y.max(), 40)
    cg = CubicGrid(X.ravel(), Y.ravel(), 40, 50)
    both = cg.interp(np.stack([F.ravel(), 2 * F.ravel()]), gx, gy).cpu().numpy()
    one = cg.interp(F.ravel(), gx, gy).cpu().numpy()[0]
    assert np.array_equal(both[0], one, equal_nan=True)
    np.testing.assert_allclose(both[1], 2 * one, rtol=1e-12, atol=1e-15)
    GH, GV = np.meshgrid(gx, gy)
    with pytest.raises(NotImplementedError):
        griddata((X.ravel(), Y.ravel()), F.ravel(), (GH, GV), method="linear")
    Xf = X.copy()
    Xf[:, 25:] = 2 * X[:, 25].reshape(-1, 1) - X[:, 25:]   # fold the lattice back on itself
    with pytest.raises(_lib.AKBError):
        CubicGrid(Xf.ravel(), Y.ravel(), 40, 50)


def _gradient_system(cg, f):
    """scipy's gradient problem on cg's triangulation in numpy: per vertex the local solve's
    Q = 4 sum r^-3 e e^T and s = sum (6 (f_i - f_j) + 2 e.g_j) r^-3 e over its edges (lattice edges by
    the cell diagonals, a ring vertex's pocket chords from xptr / xidx) as the sparse fixed-point
    problem g = c + J g (_interpnd.pyx's estimate_gradients_2d_global). Returns (J, c)."""
    import scipy.sparse as sp
    nv, nh = cg.nv, cg.nh
    x, y = cg.x.cpu().numpy(), cg.y.cpu().numpy()
    d = cg.diag.cpu().numpy().reshape(nv - 1, nh - 1).astype(bool)
    idx = np.arange(nv * nh).reshape(nv, nh)
    E = [(idx[:, :-1].ravel(), idx[:, 1:].ravel()), (idx[:-1, :].ravel(), idx[1:, :].ravel()),
         (idx[:-1, :-1][~d], idx[1:, 1:][~d]), (idx[:-1, 1:][d], idx[1:, :-1][d])]
    I = np.concatenate([e[0] for e in E])
    J = np.concatenate([e[1] for e in E])
    I, J = np.concatenate([I, J]), np.concatenate([J, I])
    xptr, xidx = cg.xptr.cpu().numpy(), cg.xidx.cpu().numpy()
    ring = np.concatenate([idx[0, :-1], idx[:-1, -1], idx[-1, :0:-1], idx[:0:-1, 0]])
    ci = np.repeat(ring, np.diff(xptr))
    I, J = np.concatenate([I, ci]), np.concatenate([J, xidx[:xptr[-1]]])
    ex, ey = x[J] - x[I], y[J] - y[I]
    r3 = (ex * ex + ey * ey) ** -1.5
    n = nv * nh
    q = [4 * np.bincount(I, w, n) for w in (ex * ex * r3, ex * ey * r3, ey * ey * r3)]
    Qi = np.linalg.inv(np.stack([np.stack([q[0], q[1]], -1), np.stack([q[1], q[2]], -1)], -2))
    w6 = 6 * (f[I] - f[J])
    s0 = np.stack([np.bincount(I, w6 * ex * r3, n), np.bincount(I, w6 * ey * r3, n)], 1)
    c = -np.einsum("nij,nj->ni", Qi, s0).ravel()
    rows, cols, vals = [], [], []
    for (a_, b_, w) in ((0, 0, ex * ex), (0, 1, ex * ey), (1, 0, ex * ey), (1, 1, ey * ey)):
        rows.append(2 * I + a_)
        cols.append(2 * J + b_)
        vals.append(2 * w * r3)
    A = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(2 * n, 2 * n))
    return -(sp.block_diag(list(Qi), format="csr") @ A), c


@pytest.mark.parametrize("nv,nh", [(97, 113), (300, 280), (33, 257)])
def test_gradient_iteration_vs_numpy_system(gpu, nv, nh):
    """The device's Chebyshev-Jacobi gradients (k_gd_sweeps + the ring chords, the edge-matrix form
    g <- c - P S) against a numpy restatement of scipy's local solve as a sparse system: five sweeps
    from zero to 1e-12 of the gradient scale (the same iteration, numpy's rounding), and converged
    (tol 1e-12) to 1e-9 of the scale of the system's direct solve; two batchings of the launches
    give the same bits."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as sla
    from akbraytracing_amd.griddata import CubicGrid, chebyshev_weights
    X, Y, F = _lattice(nv, nh, nv + nh)
    X = X * (nh / nv)
    cg = CubicGrid(X.ravel(), Y.ravel(), nv, nh)
    Jm, c = _gradient_system(cg, F.ravel())
    om = chebyshev_weights(8)
    xp, xc = np.zeros_like(c), c.copy()  # x_0 = 0, x_1 = the plain sweep
    for k in range(1, 5):
        xp, xc = xc, om[k] * (Jm @ xc + c - xp) + xp
    g5 = cg.gradients(F.ravel(), maxiter=5, check_every=5).cpu().numpy()[0].ravel()
    scale = np.max(np.abs(xc))
    assert np.max(np.abs(g5 - xc)) <= 1e-12 * scale
    assert np.array_equal(g5, cg.gradients(F.ravel(), maxiter=5, check_every=3, adaptive=False).cpu().numpy()[0].ravel())
    direct = sla.spsolve((sp.identity(c.size, format="csr") - Jm).tocsc(), c)
    gc = cg.gradients(F.ravel(), tol=1e-12, check_every=4).cpu().numpy()[0].ravel()
    assert np.max(np.abs(gc - direct)) <= 1e-9 * np.max(np.abs(direct))


def test_wave_maps_chain_vs_reference(gpu):
    """detcenter2 / Wave2 of the reference's 65x65 ray_wave run -> grid, griddata, nanmean,
    plane correction: the reference's plane_in / plane_out (= psf_calc's input)."""
    from akbraytracing_amd import pupilmap as PM
    f = golden("akb_raywave_65.npz")
    g = golden("akb_psfcalc_65.npz")
    r = PM.wave_maps(f["detcenter2"], f["dist_err2"], f["wave2"], 65, 65)
    assert np.array_equal(r["grid_H"], g["grid_H0"]) and np.array_equal(r["grid_V"], g["grid_V0"])
    w = r["matrixWave2"].cpu().numpy()
    assert np.array_equal(np.isnan(w), np.isnan(g["plane_in"]))
    rng_ = np.nanmax(g["plane_in"]) - np.nanmin(g["plane_in"])
    assert np.nanmax(np.abs(w - g["plane_in"])) <= 1e-6 * rng_
    c = r["matrixWave2_Corrected"].cpu().numpy()
    assert np.nanmax(np.abs(c - g["plane_out"])) <= 1e-6 * rng_


# ----------------------------------------------------------------------------- Huygens

def test_huygens_cases(gpu):
    from akbraytracing_amd import wavecalc as W
    h = golden("huygens_cases.npz")
    for p in "ab":
        out = W.forward_propagation_numpy_batch(h[p + "_tx"], h[p + "_ty"], h[p + "_tz"], h[p + "_sx"], h[p + "_sy"],
                                                h[p + "_sz"], h[p + "_u"], float(h[p + "_k"]), h[p + "_ds"])
        ref = h[p + "_out"]
        assert np.max(np.abs(out - ref)) <= 1e-9 * np.max(np.abs(ref)), p


def test_huygens_source_split_and_wavefield(gpu):
    """few targets x many sources (the M2 -> image stage shape) exercises the split-M path."""
    from akbraytracing_amd import wavecalc as W
    rng = np.random.default_rng(5)
    m, n = 200_000, 37
    sx, sy, sz = rng.random(m) * 1e-3, rng.random(m) * 1e-3, rng.random(m) * 1e-3
    tx, ty, tz = rng.random(n) * 1e-3, rng.random(n) * 1e-3, 0.05 + rng.random(n) * 1e-3
    u = rng.standard_normal(m) + 1j * rng.standard_normal(m)
    ds = rng.random(m)
    k = 2 * np.pi / 13.5e-9
    ref = O.huygens_c(tx, ty, tz, sx, sy, sz, u * ds, k)
    src = W.WaveField3D(m, 13.5e-9, 1, 1)
    src.setdata(np.vstack([sx, sy, sz]))
    src.set_ds(ds)
    src.u = u
    dst = W.WaveField3D(n, 13.5e-9, 1, 1)
    dst.setdata(np.vstack([tx, ty, tz]))
    dst.forward_propagation(src)
    assert np.max(np.abs(dst.u - ref)) <= 1e-9 * np.max(np.abs(ref))


def _huygens_split_case(m=400_000, n=37, seed=9):
    rng = np.random.default_rng(seed)
    s = [torch.from_numpy(rng.random(m) * 1e-3).cuda() for _ in range(3)]
    t = [torch.from_numpy(rng.random(n) * 1e-3).cuda() for _ in range(2)]
    t.append(torch.from_numpy(0.05 + rng.random(n) * 1e-3).cuda())
    u = torch.from_numpy(rng.standard_normal(m) + 1j * rng.standard_normal(m)).cuda()
    return t, s, u, 2 * np.pi / 13.5e-9


def test_huygens_nan_source_stays_fast(gpu):
    """One NaN source coordinate: every target's sum is NaN (numpy's), and the call costs about what a
    finite one does - a NaN phase stays on the fast sincos path instead of sending every target of its
    split to the library fix-up loop."""
    import time
    from akbraytracing_amd.wavecalc import propagate
    t, s, u, k = _huygens_split_case()
    clean = propagate(*t, *s, u, k)
    s_nan = [a.clone() for a in s]
    s_nan[1][12345] = float("nan")

    def timed(src):
        propagate(*t, *src, u, k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            out = propagate(*t, *src, u, k)
        torch.cuda.synchronize()
        return out, (time.perf_counter() - t0) / 5

    out, t_nan = timed(s_nan)
    _, t_ok = timed(s)
    assert torch.isnan(out.real).all() and torch.isnan(out.imag).all()
    assert torch.isfinite(clean.real).all()
    assert t_nan <= 2.0 * t_ok + 2e-3, (t_nan, t_ok)


def test_huygens_two_streams_do_not_share_scratch(gpu):
    """propagate on two streams of one thread, queued back to back so their kernels may overlap: each
    result equals the same call run alone (the split partials' scratch is per stream)."""
    from akbraytracing_amd.wavecalc import propagate
    t, s, u, k = _huygens_split_case(seed=10)
    t2 = [a.flip(0).contiguous() for a in t]
    want_a = propagate(*t, *s, u, k)
    want_b = propagate(*t2, *s, u, k)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(sa):
            got_a = propagate(*t, *s, u, k, stream=sa)
        with torch.cuda.stream(sb):
            got_b = propagate(*t2, *s, u, k, stream=sb)
        torch.cuda.synchronize()
        assert torch.equal(got_a, want_a) and torch.equal(got_b, want_b)


# ----------------------------------------------------------------------------- install

def test_install_on_a_driver_like_module(gpu):
    import types
    import akbraytracing_amd
    mod = types.ModuleType("fake_driver")
    mod.option_mpmath = False
    calls = []
    mod.mirr_ray_intersection = lambda *a, **k: calls.append("orig") or "orig"
    mod.reflect_ray = O.reflect_ray
    akbraytracing_amd.install(mod)
    d = golden("akb_primitives_33.npz")
    out = mod.mirr_ray_intersection(d["c00_mirr_ray_intersection_in0"], d["c00_mirr_ray_intersection_in1"],
                                    d["c00_mirr_ray_intersection_in2"])
    assert np.array_equal(out, d["c00_mirr_ray_intersection_out"]) and not calls
    mod.option_mpmath = True
    assert mod.mirr_ray_intersection(1, 2, 3) == "orig"
    akbraytracing_amd.uninstall(mod)
    assert mod.reflect_ray is O.reflect_ray


def test_install_runs_the_ray_wave_post_trace_chain(gpu, tmp_path):
    """The driver's :3653-3710 sequence through install()'d names: griddata x2, nanmean,
    plane correction, psf_calc reading the module's option_energy / directory_name."""
    import types
    import akbraytracing_amd
    from scipy.interpolate import griddata as sp_griddata
    mod = types.ModuleType("fake_driver")
    mod.griddata = sp_griddata
    mod.plane_correction_with_nan_and_outlier_filter = lambda m: None
    mod.psf_calc = lambda *a: None
    mod.option_energy, mod.option_AKB, mod.directory_name = "EUV", True, str(tmp_path)
    akbraytracing_amd.install(mod)
    f = golden("akb_raywave_65.npz")
    g = golden("akb_psfcalc_65.npz")
    d2 = f["detcenter2"]
    grid_H, grid_V = np.meshgrid(np.linspace(d2[1, :].min(), d2[1, :].max(), 65),
                                 np.linspace(d2[2, :].min(), d2[2, :].max(), 65))
    matrixWave2 = mod.griddata((d2[1, :], d2[2, :]), f["wave2"], (grid_H, grid_V), method="cubic")
    matrixWave2 = matrixWave2 - np.nanmean(matrixWave2)
    corrected = mod.plane_correction_with_nan_and_outlier_filter(matrixWave2)
    rng_ = np.nanmax(g["plane_out"]) - np.nanmin(g["plane_out"])
    assert np.nanmax(np.abs(corrected - g["plane_out"])) <= 1e-6 * rng_
    assert mod.psf_calc(corrected, g["grid_H"], g["grid_V"], float(g["defocus"])) is None
    assert np.load(tmp_path / "psf.npy").shape == (1056, 1056)
    akbraytracing_amd.uninstall(mod)
    assert mod.griddata is sp_griddata


# ----------------------------------------------------------------------------- large sizes

@pytest.mark.slow
def test_chain_1e6_rays_bitwise_vs_oracle(gpu):
    from akbraytracing_amd.trace import trace_chain
    g = _geom()
    n = 1001
    rh, rv = g.angle_h.table(n), g.angle_v.table(n)
    th, tv = np.tan(rh), np.tan(rv)
    res = trace_chain(g.mirrors, tan_h=torch.from_numpy(th).to(gpu), tan_v=torch.from_numpy(tv).to(gpu),
                      det_ghij=g.det1, want=("last_hit", "dir_out", "det", "opl"))
    dirs = OPL.grid_dirs(th, tv)
    mir = golden_json("akb_geometry.json")["mirrors"]
    hits, r4, segs = OPL.chain(mir, dirs, np.zeros((3, n * n)), with_segments=True)
    assert np.array_equal(res.last_hit.cpu().numpy(), hits[-1])
    assert np.array_equal(res.dir_out.cpu().numpy(), r4)
    assert np.array_equal(res.opl.cpu().numpy(), segs[0] + segs[1] + segs[2] + segs[3])


@pytest.mark.slow
def test_ray_wave_1e7_properties(gpu):
    """BASELINE config 3 size (3163^2 rays): no flags, finite OPD with zero mean, and the GPU's
    numpy-order mean of DistError2 reproduces np.nanmean of the same GPU values."""
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), 3163)
    out = rw.run()
    assert out["flags"] == (0, 0)
    w = out["wave2"].cpu().numpy()
    e = out["dist_err2"].cpu().numpy()
    assert np.isfinite(w).all() and w.shape == (3163 * 3163,)
    # numpy's own mean of 1e7 values near 146 m is good to ~1e-13 m, i.e. ~1e-4 nm of OPD
    assert abs(np.nanmean(e)) < 1e-2
    t2 = out["total2"].cpu().numpy()
    assert rw.means()[0][1] == np.nanmean(t2)
    # the OPD's spread at 1e7 rays stays within the 65^2 reference's order of magnitude (nm)
    assert 1e-4 < np.nanstd(w) < 1.0


@pytest.mark.gpu
@pytest.mark.slow
def test_psf_fft_example_at_its_own_size(gpu):
    """psf_fft_example.py unmodified in substance: `from psf_fft import compute_psf_fft` resolving
    to dropin/psf_fft.py, its 1024^2 pupil at pad_factor=16 -> 16384^2, against the reference's
    own run (tests/golden/psf_example.npz: peak, 64^2 crop, 256^2 block sums, centre row / column,
    total, axes). Tolerance: 1e-10 of the peak (rocFFT vs pocketfft rounding)."""
    import importlib
    import sys
    sys.path.insert(0, os.path.join(ROOT, "akbraytracing_amd", "dropin"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    try:
        sys.modules.pop("psf_fft", None)
        psf_fft = importlib.import_module("psf_fft")
        from make_golden_psf_example import example_inputs, summarize
    finally:
        sys.path.pop(0)
        sys.path.pop(0)
    assert psf_fft.__file__.startswith(os.path.join(ROOT, "akbraytracing_amd"))
    opd, amp, wl, dx, f = example_inputs()
    psf, x_im, y_im = psf_fft.compute_psf_fft(opd, amp, wl, dx, f, pad_factor=16, window=None)
    got = summarize(psf, x_im, y_im)
    del psf
    ref = golden("psf_example.npz")
    assert np.array_equal(got["shape"], ref["shape"]) and np.array_equal(got["peak"], ref["peak"])
    assert np.array_equal(got["x_im_sub"], ref["x_im_sub"]) and np.array_equal(got["y_im_sub"], ref["y_im_sub"])
    for k in ("crop", "row", "col"):
        assert np.max(np.abs(got[k] - ref[k])) <= 1e-10, k
    assert np.max(np.abs(got["blocks"] - ref["blocks"])) <= 1e-10 * 256 * 256
    assert abs(got["total"] - ref["total"]) <= 1e-10 * ref["total"]


@pytest.mark.parametrize("run", ["plain", "thin"])
def test_save_wave_data_files_vs_reference(gpu, tmp_path, run):
    """saveWaveData (:13475-13764) end to end at the best-alignment params on a 33 x 33 grid: the
    'wave' trace, the downsampling, calc_dS and the file writers give the reference's own files
    (tests/golden/savewave_33.npz) - every array bit for bit, the conditions text byte for byte
    (its time line set to the recorded one)."""
    from akbraytracing_amd import wavedata as W
    f = golden("savewave_33.npz")
    text = str(f[f"{run}_conditions"])
    stamp = [ln for ln in text.splitlines() if ln.startswith("time: ")][0][6:]
    folder = W.saveWaveData(golden("akb_autofocus.npz")["g0_params"], ray_num_H=33, directory=str(tmp_path / run),
                            defocus_for_wave=float(f["defocusForWave"]), downsample=tuple(f[f"{run}_downsample"]),
                            timestamp=stamp)
    for name in ("points_source", "points_M1", "points_M2", "points_M3", "points_M4", "points_gridImage",
                 "points_gridDefocus"):
        got = np.load(os.path.join(folder, name + ".npy"))
        want = f[f"{run}_{name}"]
        assert got.shape == want.shape and np.array_equal(got, want), name
    with open(os.path.join(folder, "calculation_conditions.txt")) as fh:
        assert fh.read() == text


def _subset_dirs(tan_h, tan_v, idx):
    """the reference's phai0 columns idx (flat iv * n_h + ih) without the full grid"""
    n_h = tan_h.shape[0]
    phai0 = np.zeros((3, idx.shape[0]))
    phai0[0] = 1.0
    phai0[1] = tan_h[idx % n_h]
    phai0[2] = tan_v[idx // n_h]
    return O.normalize_vector(phai0)


@pytest.mark.slow
def test_kb_wave_3163_rows_vs_oracle(gpu):
    """BASELINE config 2's trace (KB, 3163^2 = 1e7 rays, two passes): no flags, and pass 2's last
    hit, exit direction and detector hit bit-exact to the oracle on the resample picks' rays and on
    20 000 rays sampled over the whole grid (the oracle's pass 1 traced on the picks only)."""
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    gd = golden_json("kb_geometry.json")
    n = 3163
    out = RayWave(SystemGeometry.from_dict(gd), n).run(opd=False, full=True)
    assert out["flags"] == (0, 0)
    rand_h, rand_v, tan_h, tan_v = OPL.angle_tables(gd, n)
    col, v_idx, start, end, h_idx = OPL.sample_indices(n, n)
    picks = np.concatenate([h_idx, v_idx])
    _, r1, _ = OPL.chain(gd["mirrors"], _subset_dirs(tan_h, tan_v, picks), np.zeros((3, picks.shape[0])))
    nh = h_idx.shape[0]
    ah = np.arctan(r1[1, :nh] / r1[0, :nh])
    av = np.arctan(r1[2, nh:] / r1[0, nh:])
    new_h, new_v = OPL.resample_from_angles(ah, av, rand_h, rand_v)
    th2, tv2 = np.tan(new_h), np.array([np.tan(x) for x in new_v])
    rng = np.random.default_rng(11)
    idx = np.unique(np.concatenate([picks, rng.integers(0, n * n, 20000)]))
    hits, r2, _ = OPL.chain(gd["mirrors"], _subset_dirs(th2, tv2, idx), np.zeros((3, idx.shape[0])))
    det = np.zeros(10)
    det[6:10] = gd["det1"][6:10]
    d2 = O.plane_ray_intersection(det, r2, hits[-1])
    sel = torch.from_numpy(idx).to(gpu)
    assert np.array_equal(out["last_hit"][:, sel].cpu().numpy(), hits[-1])
    assert np.array_equal(out["dir_out"][:, sel].cpu().numpy(), r2)
    assert np.array_equal(out["det_pre"][:, sel].cpu().numpy(), d2)


@pytest.mark.slow
def test_huygens_c2_stage_1e7_sources(gpu):
    """BASELINE config 2's Huygens stage shape: the 1e7 last-mirror points of the KB 3163^2 run as
    sources (synthetic dS and field) -> the 65 x 65 image grid (4225 targets): the device sum
    against the oracle's C restatement on 64 sampled targets, <= 1e-9 of max |u| (the oracle walks
    all 1e7 sources for each, so only a sample)."""
    from akbraytracing_amd import wavecalc as W
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    out = RayWave(SystemGeometry.from_dict(golden_json("kb_geometry.json")), 3163).run(opd=False, full=True)
    pts = out["last_hit"].cpu().numpy()
    det = out["det_pre"].cpu().numpy()
    M = pts.shape[1]
    rng = np.random.default_rng(21)
    ds = 1e-12 * (1.0 + 0.1 * rng.random(M))
    u = np.exp(1j * 2 * np.pi * rng.random(M))
    foc = np.nanmean(det, axis=1)
    gy, gz = np.meshgrid(np.linspace(-2e-7, 2e-7, 65), np.linspace(-2e-7, 2e-7, 65))
    tx, ty, tz = np.full(4225, foc[0]), foc[1] + gy.ravel(), foc[2] + gz.ravel()
    k = 2 * np.pi / 13.5e-9
    got = W.forward_propagation_numpy_batch(tx, ty, tz, pts[0], pts[1], pts[2], u, k, ds)
    pick = rng.choice(4225, 64, replace=False)
    ref = O.huygens_c(tx[pick], ty[pick], tz[pick], pts[0], pts[1], pts[2], u * ds, k)
    assert np.max(np.abs(got[pick] - ref)) <= 1e-9 * np.max(np.abs(ref))


@pytest.mark.parametrize("n", [77, 8192, 3 * 8192 + 5, 2100 * 8192 + 2137])
def test_finish_tilt_params_fused_equals_two_calls(gpu, n):
    """akb_finish_tilt_params_f64 (one launch) = akb_leaf_finish_f64 + akb_tilt_params_f64: the
    five sums / counts and the whole parameter block bit for bit, NaNs in the nanmean rows (full
    buffers and the short one), a grid with more buffers than one LDS tile, two calls in a row."""
    from akbraytracing_amd import _lib, device as D
    from akbraytracing_amd.reduce import LeafSink
    L = _lib.lib()
    rng = np.random.default_rng(n)
    sink = LeafSink(5, n, 0b00011, gpu)
    nfull = n // 8192
    nleaves = nfull * 64
    tail = n - nfull * 8192
    for rep in range(2):
        ls = torch.from_numpy(rng.standard_normal(5 * max(nleaves, 1))[:5 * nleaves] * 1e-3).to(gpu)
        lc = torch.from_numpy(rng.integers(120, 129, 5 * nleaves).astype(np.int32)).to(gpu)
        tl = rng.standard_normal((5, 8192)) * 1e-3
        tl[2:] += 146.0
        if tail:
            tl[0, rng.integers(0, tail, 3)] = np.nan
        sink.buf.zero_()
        base = sink.buf.data_ptr()
        if nleaves:
            ptr_s = sink.desc.leaf_sum - base
            ptr_c = sink.desc.leaf_cnt - base
            sink.buf[ptr_s:ptr_s + 8 * 5 * nleaves].view(torch.float64).copy_(ls)
            sink.buf[ptr_c:ptr_c + 4 * 5 * nleaves].view(torch.int32).copy_(lc)
        pt = sink.desc.tail - base
        sink.buf[pt:pt + 8 * 5 * 8192].view(torch.float64).copy_(torch.from_numpy(tl.ravel()).to(gpu))
        # reference: the two calls
        s_ref, c_ref = (x.clone() for x in sink.finish())
        p_ref = torch.empty(25, dtype=torch.float64, device=gpu)
        keys = torch.full((4,), 7, dtype=torch.int64, device=gpu)
        fl = torch.tensor([rep + 3, 9], dtype=torch.int32, device=gpu)
        _lib.check(L.akb_tilt_params_f64(D.ptr(s_ref), D.ptr(c_ref), D.ptr(p_ref), D.ptr(keys), D.ptr(fl), 2,
                                         D.stream_handle()))
        # fused
        work = torch.empty(int(L.akb_finish_params_work_bytes(sink.desc)) // 8 + 1, dtype=torch.float64, device=gpu)
        s = torch.empty(5, dtype=torch.float64, device=gpu)
        c = torch.empty(5, dtype=torch.int64, device=gpu)
        p = torch.empty(25, dtype=torch.float64, device=gpu)
        keys2 = torch.full((4,), 7, dtype=torch.int64, device=gpu)
        fl2 = torch.tensor([rep + 3, 9], dtype=torch.int32, device=gpu)
        for _ in range(2):
            fl2.copy_(torch.tensor([rep + 3, 9], dtype=torch.int32))
            _lib.check(L.akb_finish_tilt_params_f64(sink.desc, D.ptr(s), D.ptr(c), D.ptr(p), D.ptr(keys2),
                                                    D.ptr(fl2), 2, D.ptr(work), D.stream_handle()))
            assert torch.equal(s, s_ref) and torch.equal(c, c_ref)
            assert torch.equal(p.view(torch.int64), p_ref.view(torch.int64))
        assert keys2.cpu().tolist() == [0, 0, 0, 0] and fl2.cpu().tolist() == [0, 0]
