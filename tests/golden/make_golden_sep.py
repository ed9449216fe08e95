"""Record the reference's 'sep' focus analysis (build container only; the reference never travels
to the GPU box):

    python tests/golden/make_golden_sep.py

plot_result_debug(params, 'sep') (AKB_raytrace_20250312.py:1326; the 53x53 two-pass trace of
:2849-2905, the nanmean tilt of :3565-3601) hands the tilted exit rays and last-mirror hits to
compare_sep (:9267-9560), which runs twenty coarse-to-fine plane searches (optimize_min_index
:9174-9217 over create_func_to_minimize / create_evaluation_fn :9219-9265) on row, column, partial
and diagonal ray subsets. auto_focus_sep (:12897-13318) repeats auto_focus_NA + 'sep' over five
values of one alignment parameter.

Recorded (numpy 2.2, scipy 1.15, scikit-learn as installed, float64):
  s{k}_*    'sep' runs: params, widesearch flag, compare_sep's inputs (rays, points, coeffs_det
            before the call) and its twelve outputs, coeffs_det after the call (compare_sep
            leaves the last searched plane in it).
  as{k}_*   auto_focus_sep runs: arguments, the params / 'sep' outputs of each of its five steps,
            and its return value ('abrr' vector or 'matrix' slopes). The reference's plots are
            not drawn (pyplot's savefig is a no-op while recording; no plotted value is recorded).
"""
import contextlib
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402

SEP_NAMES = ("focus_v0", "focus_h0", "pos_v0", "pos_h0", "std_v0", "std_h0", "focus_v0_l", "focus_h0_l",
             "focus_v0_u", "focus_h0_u", "focus_std_obl1", "focus_std_obl2")


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_sep_"))
    import AKB_raytrace_20250312 as A
    A.option_set = True
    A.plt.savefig = lambda *a, **k: None
    out = {}

    orig_cs = A.compare_sep
    captured = []

    def compare_sep(rays, points, coeffs_det0, ray_num, region):
        before = np.array(coeffs_det0, dtype=np.float64).copy()
        r = orig_cs(rays, points, coeffs_det0, ray_num, region)
        captured.append((np.array(rays), np.array(points), before, np.array(coeffs_det0, dtype=np.float64).copy(),
                         int(ray_num), r))
        return r
    A.compare_sep = compare_sep

    rng = np.random.default_rng(77)
    best = MG.best_params()
    scale = np.array([1e-3, 1e-4] + [1e-5, 1e-5, 1e-5, 1e-6, 1e-6, 1e-6] * 4)
    cases = [(best, False), (best + scale * rng.standard_normal(26), False),
             (best + np.r_[2e-4, -3e-4, np.zeros(24)], True)]
    for k, (p, wide) in enumerate(cases):
        A.widesearch = wide
        captured.clear()
        with contextlib.redirect_stdout(io.StringIO()):
            r = A.plot_result_debug(np.array(p, dtype=np.float64), "sep", option_save=False)
        assert len(captured) == 1
        rays, points, before, after, n, rr = captured[0]
        out[f"s{k}_params"] = np.array(p, dtype=np.float64)
        out[f"s{k}_widesearch"] = np.array(wide)
        out[f"s{k}_rays"] = rays
        out[f"s{k}_points"] = points
        out[f"s{k}_coeffs_before"] = before
        out[f"s{k}_coeffs_after"] = after
        out[f"s{k}_ray_num"] = np.array(n)
        for name, v in zip(SEP_NAMES, r):
            out[f"s{k}_{name}"] = np.array(v, dtype=np.float64)
        print("sep case", k, "focus_v0", r[0], "focus_h0", r[1])
    A.widesearch = False

    orig_prd = A.plot_result_debug
    runs = [("abrr", 9, 21, -2e-5, 2e-5, "abrr", None),
            ("matrix", 9, 21, -2e-5, 2e-5, "matrix", "9")]
    for k, (name, a1, a2, la, ua, option, oeval) in enumerate(runs):
        steps = []

        def wrapped(params, option_, *a, **kw):
            r = orig_prd(params, option_, *a, **kw)
            if option_ == "sep":
                steps.append((np.array(params, dtype=np.float64).copy(), r))
            return r
        A.plot_result_debug = wrapped
        p0 = np.array(best, dtype=np.float64)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                ret = A.auto_focus_sep(p0.copy(), a1, a2, la, ua, option=option, option_eval=oeval)
        finally:
            A.plot_result_debug = orig_prd
        out[f"as{k}_start"] = p0
        out[f"as{k}_args"] = np.array([a1, a2, la, ua], dtype=np.float64)
        out[f"as{k}_option"] = np.array(option)
        out[f"as{k}_option_eval"] = np.array("" if oeval is None else oeval)
        out[f"as{k}_step_params"] = np.stack([s[0] for s in steps])
        for j, name_ in enumerate(SEP_NAMES):
            out[f"as{k}_step_{name_}"] = np.stack([np.array(s[1][j], dtype=np.float64) for s in steps])
        out[f"as{k}_ret"] = np.array(ret, dtype=np.float64)
        print("auto_focus_sep", name, len(steps), "steps ->", ret)

    out["meta_numpy"] = np.array(np.__version__)
    np.savez_compressed(os.path.join(MG.OUT, "akb_sep.npz"), **out)
    print("wrote", os.path.join(MG.OUT, "akb_sep.npz"))


if __name__ == "__main__":
    main()
