"""KB_debug's system (the KB pair) and its focus search (row f2 with
option_AKB False) against the reference's own outputs (tests/golden/kb_build.npz, recorded by
tests/golden/make_golden_kb.py from AKB_raytrace_20250312.py itself).

CPU tests check the host logic - geometry.build_kb with the oracle's primitives standing in for the
device ones, auto_focus_NA's loop fed the recorded spot sizes - and the GPU tests the product path
end to end, bit for bit."""
import numpy as np
import pytest

from conftest import golden

KB = "kb_build.npz"
N_CASES = 7


def _case(f, k):
    d = f[f"k{k}_design"]
    return dict(params=f[f"k{k}_params"], source_shift=f[f"k{k}_source_shift"],
                designparams=None if d.size == 0 else d)


def _check_built(b, f, k):
    C = np.array([m["coeffs"] for m in b["mirrors"]])
    assert np.array_equal(C, f[f"k{k}_coeffs"]), f"case {k}: quadrics differ"
    assert [m["negative"] for m in b["mirrors"]] == [False, False]
    assert b["det1"][9] == f[f"k{k}_det_j"]


def test_kb_define_fixed_point():
    """KB_define's V ellipse shares the H ellipse's focal distance to the loop's 1e-9"""
    from akbraytracing_amd.geometry import KB_DESIGN_7PARAMS, kb_define
    a_h, b_h, a_v, b_v, l1v, l2v, rest = kb_define(*KB_DESIGN_7PARAMS)
    s2f_h = 2 * np.sqrt(a_h**2 - b_h**2)
    s2f_v = 2 * np.sqrt(a_v**2 - b_v**2)
    assert abs(s2f_h - s2f_v) < 1e-9 and rest[16] == s2f_h
    assert 0 < rest[7] < 0.1 and 0 < rest[15] < 0.1  # the two NAs


def test_build_kb_host_logic_vs_reference():
    """every case (zeros, random misalignments, pitches alone, a source shift, the paper's design
    parameters) gives the reference's two quadrics and detector plane bit for bit"""
    import oracle
    from akbraytracing_amd.geometry import build_kb
    f = golden(KB)
    for k in range(N_CASES):
        c = _case(f, k)
        b = build_kb(c["params"], source_shift=c["source_shift"], designparams=c["designparams"], prims=oracle)
        _check_built(b, f, k)


def test_build_kb_launch_grid_vs_reference():
    """the 53 x 53 launch directions of KB_debug's 'test' trace"""
    import oracle
    import oracle.pipeline as OPL
    from akbraytracing_amd.geometry import build_kb
    from akbraytracing_amd.wavefront import AngleRange
    f = golden(KB)
    for k in range(N_CASES):
        c = _case(f, k)
        b = build_kb(c["params"], source_shift=c["source_shift"], designparams=c["designparams"], prims=oracle)
        th = np.tan(AngleRange(**b["angle_h"]).table(53))
        tv = np.tan(AngleRange(**b["angle_v"]).table(53))
        assert np.array_equal(OPL.grid_dirs(th, tv), f[f"k{k}_dir0"]), f"case {k}"


def _kaf_sweeps(f):
    calls = f["kaf_calls"]
    assert len(calls) % 100 == 0
    return [calls[100 * i:100 * (i + 1)] for i in range(len(calls) // 100)]


def test_kb_auto_focus_host_loop_matches_reference_sequence():
    """auto_focus_NA with option_AKB False, fed the reference's recorded spot sizes: the same sweeps,
    astigmatism updates, answer and params left behind"""
    from akbraytracing_amd import autofocus as AFm
    f = golden(KB)
    sweeps = _kaf_sweeps(f)
    it = iter(sweeps)
    seen = []

    class FakeTS:
        def evaluate(self, a):
            blk = next(it)
            assert np.array_equal(blk[:, 0], a)
            seen.append(1)
            return blk[:, 2][None, :], blk[:, 3][None, :]

    class FakeCache:
        def get(self, params, ss, tilt):
            return FakeTS()

    p = f["kaf_start"].copy()
    ret = AFm.auto_focus_NA(50, p, 1, 1, False, "", option_AKB=False, cache=FakeCache(), verbose=False)
    assert len(seen) == len(sweeps)
    assert np.array_equal(np.array(ret[:2]), f["kaf_ret"])
    assert np.array_equal(p, f["kaf_params_after"])


# ------------------------------------------------------------------------------------------ GPU


@pytest.mark.gpu
def test_build_kb_on_device_vs_reference(gpu):
    from akbraytracing_amd.geometry import build_kb
    f = golden(KB)
    for k in range(N_CASES):
        c = _case(f, k)
        _check_built(build_kb(c["params"], source_shift=c["source_shift"], designparams=c["designparams"]), f, k)


@pytest.mark.gpu
def test_kb_test_mode_bitwise_vs_reference(gpu):
    """KB_debug(params, 1, 1, 'test'): the V hits, the tilted H hits, the tilted detector hits and
    exit directions, bit for bit, for every case"""
    from akbraytracing_amd.autofocus import kb_test
    f = golden(KB)
    for k in range(N_CASES):
        c = _case(f, k)
        r = kb_test(c["params"], c["source_shift"], designparams=c["designparams"])
        for got, name in zip(r, ("vmirr_hyp", "hmirr_hyp", "detcenter", "angle")):
            assert np.array_equal(got, f[f"k{k}_{name}"]), f"case {k}: {name} differs"


@pytest.mark.gpu
def test_kb_auto_focus_NA_bitwise_vs_reference(gpu):
    """auto_focus_NA on the KB system end to end on the device: every sweep's 100 spot sizes equal
    to the reference's 'test' calls, the same answer and params"""
    from akbraytracing_amd import autofocus as AFm
    f = golden(KB)
    sweeps = _kaf_sweeps(f)
    log = []

    class LoggingCache(AFm._SystemCache):
        def get(self, params, ss, tilt):
            ts = super().get(params, ss, tilt)

            class Wrap:
                def evaluate(self_inner, a):
                    sv, sh = ts.evaluate(a)
                    log.append((np.array(a), float(params[1]), sv[0].copy(), sh[0].copy()))
                    return sv, sh
            return Wrap()

    p = f["kaf_start"].copy()
    ret = AFm.auto_focus_NA(50, p, 1, 1, False, "", option_AKB=False, cache=LoggingCache(True, 53, "kb"),
                            verbose=False)
    assert np.array_equal(np.array(ret[:2]), f["kaf_ret"])
    assert len(log) == len(sweeps)
    for i, ((a, p1, sv, sh), blk) in enumerate(zip(log, sweeps)):
        assert np.array_equal(a, blk[:, 0])
        assert np.all(blk[:, 1] == p1)
        assert np.array_equal(sv, blk[:, 2]), f"sweep {i}: size_v differs"
        assert np.array_equal(sh, blk[:, 3]), f"sweep {i}: size_h differs"
    assert np.array_equal(p, f["kaf_params_after"])


@pytest.mark.gpu
def test_install_routes_kb_debug_and_kb_auto_focus(gpu):
    """install(): KB_debug(params, ..., 'test') and auto_focus_NA with option_AKB False run on the
    device; KB_debug's other modes stay the module's own"""
    import types
    import akbraytracing_amd
    f = golden(KB)
    mod = types.ModuleType("fake_driver")
    mod.option_AKB, mod.option_wolter_3_1, mod.option_mpmath = False, True, False
    mod.option_set, mod.widesearch = True, False
    seen = []
    mod.plot_result_debug = lambda params, option, **kw: seen.append(option) or "orig"
    mod.KB_debug = lambda params, na_h, na_v, option, **kw: seen.append("kb-" + option) or "orig-kb"
    mod.auto_focus_NA = lambda *a, **kw: seen.append("af") or "orig-af"
    akbraytracing_amd.install(mod)
    try:
        r = mod.KB_debug(f["k0_params"], 1, 1, "test")
        assert np.array_equal(r[2], f["k0_detcenter"]) and not seen
        assert mod.KB_debug(f["k0_params"], 1, 1, "ray") == "orig-kb" and seen == ["kb-ray"]
        p = f["kaf_start"].copy()
        ret = mod.auto_focus_NA(50, p, 1, 1, False, "")
        assert np.array_equal(np.array(ret[:2]), f["kaf_ret"]) and np.array_equal(p, f["kaf_params_after"])
    finally:
        akbraytracing_amd.uninstall(mod)
    assert mod.KB_debug(f["k0_params"], 1, 1, "test") == "orig-kb"


def test_kb_ray_wave_conditions():
    from akbraytracing_amd.driver import kb_ray_wave_conditions
    assert kb_ray_wave_conditions() == (1e-4, 13.5)
    assert kb_ray_wave_conditions(True, "hardXray", True) == (1e-1, 0.135)
    assert kb_ray_wave_conditions(False, "hardXray") == (1e-5, 1.35)
    with pytest.raises(ValueError):
        kb_ray_wave_conditions(True, "visible")


@pytest.mark.gpu
@pytest.mark.parametrize("c", [0, 1, 2])
def test_kb_ray_wave_vs_reference(gpu, tmp_path, c):
    """KB_debug(params, 1, 1, 'ray_wave', option_legendre=True) on the device: the griddata points
    and values, the corrected map psf_calc receives (tests/golden/kb_raywave.npz, recorded from the
    reference), then the rectification (256 x 256) and Legendre fit against the oracle's
    composition on the reference's own map; the files the mode writes"""
    import oracle.affine as OA
    import oracle.legendre as OLg
    from akbraytracing_amd.driver import kb_ray_wave
    g = golden("kb_raywave.npz")
    n = int(g[f"c{c}_n"])
    out_dir = tmp_path / "out"
    r = kb_ray_wave(g[f"c{c}_params"], n, directory=str(out_dir), workdir=str(tmp_path), verbose=False, as_dict=True)
    run = r["run"]
    det2 = run["detcenter2"].cpu().numpy()[1:3]
    want = g[f"c{c}_det2"]
    # the tilt's angles are the reference's to an ulp of arctan (DESIGN a7)
    assert np.max(np.abs(det2 - want)) <= 1e-12 * np.max(np.ptp(want, axis=1))
    w = run["wave2"].cpu().numpy()
    ref_w = g[f"c{c}_wave2"]
    assert np.max(np.abs(w - ref_w)) <= 1e-6 * np.ptp(ref_w)
    corr = r["maps"]["matrixWave2_Corrected"].cpu().numpy()
    ref = g[f"c{c}_plane_out"]
    assert np.array_equal(np.isnan(corr), np.isnan(ref))
    assert np.nanmax(np.abs(corr - ref)) <= 1e-6 * (np.nanmax(ref) - np.nanmin(ref))
    # past psf_calc: cv2's step is unpinned (absent here); the oracle's composition on the
    # reference's map
    rect = OA.extract_affine_square_region(ref / 13.5, target_size=256)
    assert r["rectified_img"].shape == (256, 256)
    assert np.array_equal(np.isnan(r["rectified_img"]), np.isnan(rect))
    assert np.nanmax(np.abs(r["rectified_img"] - rect)) <= 1e-6 * np.nanmax(np.abs(rect))
    fits, ip = OLg.fit_multi(rect[1:-2, 1:-2], 5)
    assert np.max(np.abs(r["inner_products"] - ip)) <= 1e-6 * np.max(np.abs(ip))
    for name in ("psf.npy", "matrixWave2_Corrected(lambda).txt", "rectified_img.txt", "inner_products.txt",
                 "orders.txt", "pvs.txt", "fit_sum.txt", "pv.txt"):
        assert (out_dir / name).exists(), name
    assert (tmp_path / "matrixWave2(nm).txt").exists()
    # pvs.txt is written before the last entry is set (:11866, :11878)
    saved = np.loadtxt(out_dir / "pvs.txt")
    assert saved[-1] == 0.0 and np.array_equal(saved[:-1], r["pvs"][:-1])
    assert r["pvs"][-1] == np.nanstd(corr / 13.5) * 6 * np.sign(np.sum(r["inner_products"]))


@pytest.mark.gpu
def test_install_routes_kb_ray_wave(gpu, tmp_path, monkeypatch):
    import types
    import akbraytracing_amd
    monkeypatch.chdir(tmp_path)
    g = golden("kb_raywave.npz")
    mod = types.ModuleType("fake_driver")
    mod.option_AKB, mod.option_mpmath, mod.option_HighNA, mod.option_energy = False, False, True, "EUV"
    mod.wave_num_H = mod.wave_num_V = 33
    mod.directory_name = str(tmp_path / "d")
    seen = []
    mod.KB_debug = lambda params, na_h, na_v, option, **kw: seen.append(option) or "orig-kb"
    akbraytracing_amd.install(mod)
    try:
        ip, orders, pvs = mod.KB_debug(g["c2_params"], 1, 1, "ray_wave", option_legendre=True)
        assert not seen and len(ip) == 15 and len(pvs) == 16
        pv = mod.KB_debug(g["c2_params"], 1, 1, "ray_wave")
        assert np.isfinite(pv) and (tmp_path / "d" / "optical_params.txt").exists()
        assert mod.KB_debug(g["c2_params"], 1, 1, "ray_wave", option_save=False) == "orig-kb"
    finally:
        akbraytracing_amd.uninstall(mod)


@pytest.mark.gpu
def test_kb_c2_pipeline_vs_oracle(gpu):
    """bench.py --config c2's system (KB_debug's pair at params = 0, second plane at defocusForWave)
    through RayWave - pass 1, resample, pass 2, tilt, OPD - against the oracle's pipeline on the
    same geometry: resampled tables bitwise, the hits and OPD to the tilt's ulp"""
    import oracle.pipeline as OPL
    import bench
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    g = bench.geometry_dict("c2")
    ref = OPL.akb_ray_wave(g, 65)
    out = RayWave(SystemGeometry.from_dict(g), 65).run(keep_rotated=True, full=True)
    assert out["flags"] == (0, 0)
    assert np.array_equal(out["tan_h2"].cpu().numpy(), ref["tan_h2"])
    assert np.array_equal(out["last_hit"].cpu().numpy(), ref["hits"][-1])
    for key in ("detcenter", "detcenter2"):
        got, want = out[key].cpu().numpy(), ref[key]
        assert np.max(np.abs(got - want)) <= 64 * np.max(np.spacing(np.abs(want))), key
    for key in ("dist_err2", "wave2"):
        assert np.max(np.abs(out[key].cpu().numpy() - ref[key])) <= 1e-4, key


@pytest.mark.gpu
def test_kb_wave_mode_bitwise_vs_reference(gpu):
    """KB_debug(params, 1, 1, 'wave') at 33 x 33: the rotated source, mirror grids, both detector
    planes, the mirror normals and the segment directions, bit for bit
    (tests/golden/kb_savewave_33.npz)"""
    from akbraytracing_amd.wavedata import kb_wave
    f = golden("kb_savewave_33.npz")
    r = kb_wave(f["params"], 33, defocus_for_wave=float(f["defocusForWave"]))
    names = ("source", "vmirr_hyp", "hmirr_hyp", "detcenter", "detcenter2", "ray_num_H", "ray_num_V", "vmirr_norm",
             "hmirr_norm", "vec0to1", "vec1to2")
    assert len(r) == len(names)
    for name, got in zip(names, r):
        assert np.array_equal(np.asarray(got), f[f"w_{name}"]), name


@pytest.mark.gpu
@pytest.mark.parametrize("run", ["plain", "thin"])
def test_kb_save_wave_data_files_vs_reference(gpu, tmp_path, run):
    """saveWaveData with option_AKB False (:13483-13487): KB 'wave', downsampling, calc_dS and the
    two-mirror file set - every array bit for bit, the conditions text byte for byte"""
    import os
    from akbraytracing_amd import wavedata as W
    f = golden("kb_savewave_33.npz")
    text = str(f[f"{run}_conditions"])
    stamp = [ln for ln in text.splitlines() if ln.startswith("time: ")][0][6:]
    folder = W.saveWaveData(f["params"], ray_num_H=33, directory=str(tmp_path / run),
                            defocus_for_wave=float(f["defocusForWave"]), downsample=tuple(f[f"{run}_downsample"]),
                            timestamp=stamp, option_AKB=False)
    for name in ("points_source", "points_M1", "points_M2", "points_gridImage", "points_gridDefocus"):
        got = np.load(os.path.join(folder, name + ".npy"))
        want = f[f"{run}_{name}"]
        assert got.shape == want.shape and np.array_equal(got, want), name
    assert not os.path.exists(os.path.join(folder, "points_M3.npy"))
    with open(os.path.join(folder, "calculation_conditions.txt")) as fh:
        assert fh.read() == text


@pytest.mark.gpu
def test_install_routes_kb_wave(gpu):
    import types
    import akbraytracing_amd
    f = golden("kb_savewave_33.npz")
    mod = types.ModuleType("fake_driver")
    mod.option_AKB, mod.option_mpmath, mod.option_rotate, mod.option_avrgsplt = False, False, True, False
    mod.wave_num_H = mod.wave_num_V = 33
    mod.defocusForWave = float(f["defocusForWave"])
    mod.KB_debug = lambda *a, **kw: "orig-kb"
    akbraytracing_amd.install(mod)
    try:
        r = mod.KB_debug(f["params"], 1, 1, "wave")
        assert np.array_equal(r[4], f["w_detcenter2"])
        mod.option_avrgsplt = True  # the split-average variant is not restated
        assert mod.KB_debug(f["params"], 1, 1, "wave") == "orig-kb"
    finally:
        akbraytracing_amd.uninstall(mod)
