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
