"""Record the reference's 'sep' focus analysis of KB_debug's pair (build container only; the
reference never travels to the GPU box):

    python tests/golden/make_golden_kb_sep.py

KB_debug(params, 1, 1, 'sep') (AKB_raytrace_20250312.py:9742; the 53x53 trace, reset_p0's
equal-angle resample :11001-11054, the np.mean tilt :11703-11717) hands the tilted exit rays and
H-mirror hits to compare_sep (:9267-9560, :11719-11721). auto_focus_sep (:12897-13318) with
option_AKB False repeats auto_focus_NA + KB_debug 'sep' (:12903, :13024) and returns the KB
measure set (:12978, :13158).

Recorded (numpy 2.2, scikit-learn as installed, float64):
  s{k}_*    'sep' runs: params, widesearch flag, the twelve outputs, coeffs_det after the call
  as{k}_*   auto_focus_sep runs: arguments, the params and 'sep' outputs of each step, the return
"""
import contextlib
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402
from make_golden_sep import SEP_NAMES  # noqa: E402


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_kbsep_"))
    import AKB_raytrace_20250312 as A
    A.plt.savefig = lambda *a, **k: None
    A.option_AKB = False
    out = {}
    orig_cs = A.compare_sep
    captured = []

    def compare_sep(rays, points, coeffs_det0, ray_num, region):
        r = orig_cs(rays, points, coeffs_det0, ray_num, region)
        captured.append(np.array(coeffs_det0, dtype=np.float64).copy())
        return r
    A.compare_sep = compare_sep
    rng = np.random.default_rng(78)
    scale = np.array([1e-3, 1e-4] + [1e-5, 1e-5, 1e-5, 1e-6, 1e-6, 1e-6] * 2 + [0.0] * 12)
    p1 = np.zeros(26)
    p1[0], p1[1] = 2e-3, -1e-4
    cases = [(np.zeros(26), False), (scale * rng.standard_normal(26), False), (p1, True)]
    for k, (p, wide) in enumerate(cases):
        A.widesearch = wide
        captured.clear()
        with contextlib.redirect_stdout(io.StringIO()):
            r = A.KB_debug(np.array(p, dtype=np.float64), 1, 1, "sep", option_save=False)
        assert len(captured) == 1
        out[f"s{k}_params"] = np.array(p, dtype=np.float64)
        out[f"s{k}_widesearch"] = np.array(wide)
        out[f"s{k}_coeffs_after"] = captured[0]
        for name, v in zip(SEP_NAMES, r):
            out[f"s{k}_{name}"] = np.array(v, dtype=np.float64)
        print("KB sep case", k, "focus_v0", r[0], "focus_h0", r[1])
    A.widesearch = False

    orig_kb = A.KB_debug
    start = np.zeros(26)
    start[0], start[1] = 2e-3, -1e-4
    runs = [(2, 2, -2e-5, 2e-5, "abrr", None), (2, 2, -2e-5, 2e-5, "matrix", None)]
    for k, (a1, a2, la, ua, option, oeval) in enumerate(runs):
        steps = []

        def wrapped(params, na_h, na_v, option_, *a, **kw):
            r = orig_kb(params, na_h, na_v, option_, *a, **kw)
            if option_ == "sep":
                steps.append((np.array(params, dtype=np.float64).copy(), r))
            return r
        A.KB_debug = wrapped
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                ret = A.auto_focus_sep(start.copy(), a1, a2, la, ua, option=option, option_eval=oeval)
        finally:
            A.KB_debug = orig_kb
        out[f"as{k}_start"] = start.copy()
        out[f"as{k}_args"] = np.array([a1, a2, la, ua], dtype=np.float64)
        out[f"as{k}_option"] = np.array(option)
        out[f"as{k}_option_eval"] = np.array("" if oeval is None else oeval)
        out[f"as{k}_step_params"] = np.stack([s[0] for s in steps])
        for j, name_ in enumerate(SEP_NAMES):
            out[f"as{k}_step_{name_}"] = np.stack([np.array(s[1][j], dtype=np.float64) for s in steps])
        out[f"as{k}_ret"] = np.array(ret, dtype=np.float64)
        print("KB auto_focus_sep", option, len(steps), "steps ->", ret)
    A.option_AKB = True
    out["meta_numpy"] = np.array(np.__version__)
    np.savez_compressed(os.path.join(MG.OUT, "kb_sep.npz"), **out)
    print("wrote", os.path.join(MG.OUT, "kb_sep.npz"))


if __name__ == "__main__":
    main()
