"""plot_result_debug's 'sep' analysis, compare_sep and auto_focus_sep (row f2) against the
reference's own outputs (tests/golden/akb_sep.npz, recorded by tests/golden/make_golden_sep.py from
AKB_raytrace_20250312.py itself).

CPU tests pin the oracle's restatement (oracle/sep.py) and the host logic (the twenty subsets, the
auto_focus_sep measures and fits); GPU tests run the product path - akb_sep_search_f64, the
two-pass 'sep' trace, auto_focus_sep over the native auto_focus_NA - bit for bit."""
import numpy as np
import pytest

from conftest import golden

SEP = "akb_sep.npz"
N_SEP = 3


def _outputs(f, pre):
    from akbraytracing_amd.sep import SEP_OUTPUTS
    return [f[f"{pre}_{k}"] for k in SEP_OUTPUTS]


def _check(r, f, pre):
    from akbraytracing_amd.sep import SEP_OUTPUTS
    for name, got, want in zip(SEP_OUTPUTS, r, _outputs(f, pre)):
        assert np.array_equal(np.asarray(got), want), f"{pre}: {name} differs: {got} vs {want}"


def test_sep_subsets_match_the_reference_index_sets():
    """(start, step, count) of every search equals the reference's index lists (odd / even grids,
    the [:-0] empty case, diagonals over any ray count)"""
    import oracle.sep as OS
    from akbraytracing_amd.sep import sep_subsets
    for n, nr in [(2, 4), (3, 9), (4, 16), (5, 25), (53, 2809), (54, 2916), (65, 4225), (7, 40)]:
        got = sep_subsets(n, nr)
        want = OS.subsets(n, nr)
        assert len(got) == len(want) == 20
        for (s, st, c), w in zip(got, want):
            assert list(s + st * np.arange(c)) == list(np.asarray(w, dtype=np.int64)), (n, nr, s, st, c)


def test_oracle_compare_sep_vs_reference():
    """the oracle's compare_sep (C plane intersections + numpy std) reproduces the reference's
    twelve outputs and its left-behind coeffs_det bit for bit, widesearch included"""
    import oracle.sep as OS
    f = golden(SEP)
    for k in range(N_SEP):
        c = f[f"s{k}_coeffs_before"].copy()
        r = OS.compare_sep(f[f"s{k}_rays"], f[f"s{k}_points"], c, int(f[f"s{k}_ray_num"]),
                           widesearch=bool(f[f"s{k}_widesearch"]))
        _check(r, f, f"s{k}")
        assert np.array_equal(c, f[f"s{k}_coeffs_after"])


@pytest.mark.parametrize("k", [0, 1])
def test_sep_summary_vs_reference(k):
    """auto_focus_sep's measures from its recorded 'sep' steps: the 'abrr' vector and the 'matrix'
    slopes (scikit-learn fits) equal the reference's returns"""
    from akbraytracing_amd.sep import SEP_OUTPUTS, _ABRR_SETS, _abrr, sep_summary
    f = golden(SEP)
    pre = f"as{k}"
    steps = [[f[f"{pre}_step_{name}"][j] for name in SEP_OUTPUTS] for j in range(len(f[f"{pre}_step_params"]))]
    for j in range(len(steps)):
        steps[j][10], steps[j][11] = np.float64(steps[j][10]), np.float64(steps[j][11])
    option = str(f[f"{pre}_option"])
    oeval = str(f[f"{pre}_option_eval"]) or None
    if option == "abrr":
        m = _abrr(steps[0])
        got = np.array([m[key] for key in _ABRR_SETS.get(oeval, _ABRR_SETS["9"]).split()])
    else:
        a1, a2, la, ua = f[f"{pre}_args"]
        p0 = f[f"{pre}_start"]
        a_param = np.linspace(la, ua, 5) + (p0[int(a1)] + p0[int(a2)]) / 2
        got = sep_summary(a_param, np.zeros(5), steps, option, oeval, verbose=False)
    assert np.array_equal(got, f[f"{pre}_ret"])


@pytest.mark.gpu
def test_compare_sep_bitwise_vs_reference(gpu):
    """akb_sep_search_f64 on the reference's own compare_sep inputs: all twenty searches (best
    plane, its spot size), the hit means on the last plane and the coeffs_det it leaves behind"""
    from akbraytracing_amd.sep import compare_sep
    f = golden(SEP)
    for k in range(N_SEP):
        c = f[f"s{k}_coeffs_before"].copy()
        r = compare_sep(f[f"s{k}_rays"], f[f"s{k}_points"], c, int(f[f"s{k}_ray_num"]), 1e-4,
                        widesearch=bool(f[f"s{k}_widesearch"]), verbose=False)
        _check(r, f, f"s{k}")
        assert np.array_equal(c, f[f"s{k}_coeffs_after"])


@pytest.mark.gpu
def test_compare_sep_device_vs_oracle_random(gpu):
    """random ray bundles around a focus (odd and even grids, a NaN ray): device == oracle"""
    import oracle.sep as OS
    from akbraytracing_amd.sep import compare_sep
    rng = np.random.default_rng(5)
    for n in (9, 20, 53):
        N = n * n
        d = np.vstack([np.ones(N), 1e-3 * rng.standard_normal(N), 1e-3 * rng.standard_normal(N)])
        d /= np.sqrt((d[0] ** 2 + d[1] ** 2) + d[2] ** 2)
        p = np.vstack([np.full(N, 10.0), 1e-3 * rng.standard_normal(N), 1e-3 * rng.standard_normal(N)])
        if n == 20:
            d[1, 7] = np.nan
        c0 = np.zeros(10)
        c0[6], c0[9] = 1.0, -10.0 - 0.003 * rng.standard_normal()
        c1, c2 = c0.copy(), c0.copy()
        want = OS.compare_sep(d, p, c1, n)
        got = compare_sep(d, p, c2, n, 1e-4, verbose=False)
        for a, b in zip(got, want):
            assert np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True), n
        assert np.array_equal(c1, c2)


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(N_SEP))
def test_plot_result_sep_bitwise_vs_reference(gpu, k):
    """plot_result_debug(params, 'sep') end to end: two-pass trace, nanmean tilt, compare_sep"""
    from akbraytracing_amd.sep import plot_result_sep
    f = golden(SEP)
    r = plot_result_sep(f[f"s{k}_params"], widesearch=bool(f[f"s{k}_widesearch"]), verbose=False)
    _check(r, f, f"s{k}")


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1])
def test_auto_focus_sep_bitwise_vs_reference(gpu, k):
    """auto_focus_sep over the native auto_focus_NA and 'sep': every step's focused params and
    'sep' outputs, and the 'abrr' / 'matrix' return"""
    from akbraytracing_amd import sep as S
    f = golden(SEP)
    pre = f"as{k}"
    seen = []
    orig = S.plot_result_sep

    def logging(p, **kw):
        r = orig(p, **kw)
        seen.append((np.array(p).copy(), r))
        return r
    S.plot_result_sep = logging
    try:
        a1, a2, la, ua = f[f"{pre}_args"]
        oeval = str(f[f"{pre}_option_eval"]) or None
        ret = S.auto_focus_sep(f[f"{pre}_start"].copy(), int(a1), int(a2), la, ua, option=str(f[f"{pre}_option"]),
                               option_eval=oeval, verbose=False)
    finally:
        S.plot_result_sep = orig
    assert len(seen) == len(f[f"{pre}_step_params"])
    for j, (p, r) in enumerate(seen):
        assert np.array_equal(p, f[f"{pre}_step_params"][j]), f"step {j}: focused params differ"
        for name, got in zip(S.SEP_OUTPUTS, r):
            assert np.array_equal(np.asarray(got), f[f"{pre}_step_{name}"][j]), f"step {j}: {name} differs"
    assert np.array_equal(ret, f[f"{pre}_ret"])


@pytest.mark.gpu
def test_install_rebinds_sep_mode_and_compare_sep(gpu):
    """install(): plot_result_debug(params, 'sep') and compare_sep go to the device, reading the
    module's live widesearch flag"""
    import types
    import akbraytracing_amd
    f = golden(SEP)
    mod = types.ModuleType("fake_driver")
    mod.option_AKB, mod.option_wolter_3_1, mod.option_mpmath = True, True, False
    mod.option_set, mod.widesearch = True, False
    mod.plot_result_debug = lambda params, option, **kw: "orig"
    mod.compare_sep = lambda *a: "orig"
    akbraytracing_amd.install(mod)
    try:
        mod.widesearch = bool(f["s2_widesearch"])
        _check(mod.plot_result_debug(f["s2_params"], "sep"), f, "s2")
        c = f["s0_coeffs_before"].copy()
        mod.widesearch = False
        _check(mod.compare_sep(f["s0_rays"], f["s0_points"], c, 53, 1e-4), f, "s0")
    finally:
        akbraytracing_amd.uninstall(mod)
    assert mod.compare_sep() == "orig"
