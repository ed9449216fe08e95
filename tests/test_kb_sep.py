"""KB_debug's 'sep' analysis and auto_focus_sep with option_AKB False (row f2 on the KB pair)
against the reference's own outputs (tests/golden/kb_sep.npz, recorded by
tests/golden/make_golden_kb_sep.py from AKB_raytrace_20250312.py itself).

The CPU test checks the host measures (the KB measure set a0, a2, a4) from the recorded steps; the
GPU tests run the product path - build_kb, the two-pass trace, the np.mean tilt, compare_sep in one
launch, auto_focus_NA's KB sweeps - bit for bit."""
import numpy as np
import pytest

from conftest import golden

KS = "kb_sep.npz"


def _check(r, f, pre):
    from akbraytracing_amd.sep import SEP_OUTPUTS
    for name, got in zip(SEP_OUTPUTS, r):
        assert np.array_equal(np.asarray(got), f[f"{pre}_{name}"]), f"{pre}: {name} differs"


def _steps(f, pre):
    from akbraytracing_amd.sep import SEP_OUTPUTS
    steps = [[f[f"{pre}_step_{name}"][j] for name in SEP_OUTPUTS] for j in range(len(f[f"{pre}_step_params"]))]
    for s in steps:
        s[10], s[11] = np.float64(s[10]), np.float64(s[11])
    return steps


@pytest.mark.parametrize("k", [0, 1])
def test_kb_sep_summary_vs_reference(k):
    """auto_focus_sep's KB returns from its recorded 'sep' steps: the 'abrr' vector (a0, a2, a4)
    and the 'matrix' slopes (scikit-learn fits, KB set)"""
    from akbraytracing_amd.sep import _ABRR_SETS, _abrr, sep_summary
    f = golden(KS)
    pre = f"as{k}"
    steps = _steps(f, pre)
    option = str(f[f"{pre}_option"])
    if option == "abrr":
        m = _abrr(steps[0])
        got = np.array([m[key] for key in _ABRR_SETS["KB"].split()])
    else:
        a1, a2, la, ua = f[f"{pre}_args"]
        p0 = f[f"{pre}_start"]
        a_param = np.linspace(la, ua, 5) + (p0[int(a1)] + p0[int(a2)]) / 2
        got = sep_summary(a_param, np.zeros(5), steps, option, None, verbose=False, option_AKB=False)
    assert np.array_equal(got, f[f"{pre}_ret"])


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1, 2])
def test_kb_sep_bitwise_vs_reference(gpu, k):
    """KB_debug(params, 1, 1, 'sep') end to end: build_kb, two-pass trace, np.mean tilt, compare_sep"""
    from akbraytracing_amd.sep import kb_sep
    f = golden(KS)
    r = kb_sep(f[f"s{k}_params"], widesearch=bool(f[f"s{k}_widesearch"]), verbose=False)
    _check(r, f, f"s{k}")


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1])
def test_kb_auto_focus_sep_bitwise_vs_reference(gpu, k):
    """auto_focus_sep with option_AKB False over the native KB auto_focus_NA and kb_sep: every
    step's focused params and 'sep' outputs, and the 'abrr' / 'matrix' return"""
    from akbraytracing_amd import sep as S
    f = golden(KS)
    pre = f"as{k}"
    seen = []
    orig = S.kb_sep

    def logging(p, **kw):
        r = orig(p, **kw)
        seen.append((np.array(p).copy(), r))
        return r
    S.kb_sep = logging
    try:
        a1, a2, la, ua = f[f"{pre}_args"]
        ret = S.auto_focus_sep(f[f"{pre}_start"].copy(), int(a1), int(a2), la, ua, option=str(f[f"{pre}_option"]),
                               option_AKB=False, verbose=False)
    finally:
        S.kb_sep = orig
    assert len(seen) == len(f[f"{pre}_step_params"])
    for j, (p, r) in enumerate(seen):
        assert np.array_equal(p, f[f"{pre}_step_params"][j]), f"step {j}: focused params differ"
        for name, got in zip(S.SEP_OUTPUTS, r):
            assert np.array_equal(np.asarray(got), f[f"{pre}_step_{name}"][j]), f"step {j}: {name} differs"
    assert np.array_equal(ret, f[f"{pre}_ret"])


@pytest.mark.gpu
def test_install_routes_kb_sep(gpu):
    """install(): KB_debug(params, 1, 1, 'sep') goes to the device with the module's widesearch"""
    import types
    import akbraytracing_amd
    f = golden(KS)
    mod = types.ModuleType("fake_driver")
    mod.option_AKB, mod.option_mpmath, mod.widesearch = False, False, True
    mod.KB_debug = lambda *a, **kw: "orig-kb"
    mod.compare_sep = lambda *a, **kw: "orig-cs"
    akbraytracing_amd.install(mod)
    try:
        _check(mod.KB_debug(f["s2_params"], 1, 1, "sep"), f, "s2")
    finally:
        akbraytracing_amd.uninstall(mod)
