"""Record the reference's system construction and focus search (build container only; the reference
never travels to the GPU box):

    python tests/golden/make_golden_autofocus.py

plot_result_debug (AKB_raytrace_20250312.py:1326, the Wolter III+I Setting12 / setting11 system
of :1706-1755) turns params[26] into four quadrics (:1902-2427, misalignment :2458-2673) before it
traces; auto_focus_NA (:12746-12895) calls it in 'test' mode hundreds of times with params[0]
(the detector defocus) swept. Recorded per case, by wrapping the reference's own module-level
primitives (resolved through globals at call time):

  g{k}_*   geometry cases: params, option_set, source_shift -> the four 53x53-ray quadrics in
           trace order, root signs, the detector plane's j (coeffs_det[9]), the launch
           directions / source of mirror 1, and the 'test' return's np.std of detcenter rows
           (tilted, and untilted with option_tilt=False). Cases 0 and 2 also keep the full
           'test' return (four hit arrays, detcenter, angle).
  af{k}_*  auto_focus_NA runs: the start params, the sequence of (params[0], params[1], std_v,
           std_h) over every 'test' call it makes, and its return value.

Writes akb_autofocus.npz (numpy 2.2, scipy 1.15, float64).
"""
import contextlib
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402

N53 = 53 * 53


def geometry_cases():
    """(params, option_set, source_shift) triples covering every misalignment entry."""
    rng = np.random.default_rng(2026)
    best = MG.best_params()
    cases = [(best, True, [0.0, 0.0, 0.0]), (np.zeros(26), True, [0.0, 0.0, 0.0])]
    # every entry perturbed: angles (pitch / roll / yaw) ~1e-5 rad, decenters ~1e-6 m
    scale = np.array([1e-3, 1e-4] + [1e-5, 1e-5, 1e-5, 1e-6, 1e-6, 1e-6] * 4)
    for k in range(3):
        p = best + scale * rng.standard_normal(26)
        cases.append((p, True, [0.0, 0.0, 0.0]))
    p = best + scale * rng.standard_normal(26)
    cases.append((p, False, [0.0, 0.0, 0.0]))            # option_set=False: per-mirror centres
    cases.append((best.copy(), True, [0.0, 2e-3, -1e-3]))  # source shift (calc_FoC, :13782)
    p = best.copy()
    p[2], p[14] = 2e-5, -1e-5                               # V pitch only (hyp reference + relative)
    cases.append((p, True, [0.0, 0.0, 0.0]))
    return cases


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_af_"))
    import AKB_raytrace_20250312 as A
    out = {}

    def run_test(p, source_shift, tilt):
        rec = MG.Recorder(A)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                r = A.plot_result_debug(np.array(p, dtype=np.float64), "test", source_shift=list(source_shift),
                                        option_tilt=tilt, option_save=False)
        finally:
            rec.restore()
        return rec.calls, r

    for k, (p, oset, ss) in enumerate(geometry_cases()):
        A.option_set = oset
        calls, r = run_test(p, ss, True)
        big = MG.big(calls, N53)
        isects = [c for c in big if c[0] == "mirr_ray_intersection"]
        planes = [c for c in big if c[0] == "plane_ray_intersection"]
        assert len(isects) == 4, len(isects)
        out[f"g{k}_params"] = np.array(p, dtype=np.float64)
        out[f"g{k}_option_set"] = np.array(oset)
        out[f"g{k}_source_shift"] = np.array(ss, dtype=np.float64)
        out[f"g{k}_coeffs"] = np.stack([c[1][0] for c in isects])
        out[f"g{k}_negative"] = np.array([bool(c[2].get("negative", False)) for c in isects])
        out[f"g{k}_det_j"] = np.float64(planes[0][1][0][9])
        if k in (0, 6):
            out[f"g{k}_dir0"] = isects[0][1][1]
            out[f"g{k}_src0"] = isects[0][1][2]
        det, ang = r[4], r[5]
        out[f"g{k}_std"] = np.array([np.std(det[2, :]), np.std(det[1, :])])
        _, r0 = run_test(p, ss, False)
        out[f"g{k}_std_notilt"] = np.array([np.std(r0[4][2, :]), np.std(r0[4][1, :])])
        if k in (0, 2):
            out[f"g{k}_hits"] = np.stack([r[0], r[2], r[3], r[1]])  # trace order: V hyp, V ell, H ell, H hyp
            out[f"g{k}_detcenter"] = det
            out[f"g{k}_angle"] = ang
            out[f"g{k}_detcenter_notilt"] = r0[4]
        print("geometry case", k, "std", out[f"g{k}_std"])

    # auto_focus_NA runs: every 'test' call recorded
    A.option_set = True
    orig = A.plot_result_debug
    runs = [
        ("best", MG.best_params(), "", False, [0.0, 0.0, 0.0]),
        ("astig", MG.best_params() + np.r_[3e-4, -2e-4, np.zeros(24)], "", False, [0.0, 0.0, 0.0]),
        ("foc", MG.best_params(), "FoC", "FoC", [0.0, 2e-3, -1e-3]),
    ]
    for k, (name, p0, oparam, omode, ss) in enumerate(runs):
        log = []

        def wrapped(params, option, **kw):
            r = orig(params, option, **kw)
            if option == "test":
                log.append((params[0], params[1], np.std(r[4][2, :]), np.std(r[4][1, :])))
            return r
        A.plot_result_debug = wrapped
        start = np.array(p0, dtype=np.float64)
        live = start.copy()
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                ret = A.auto_focus_NA(50, live, 1, 1, oparam == "FoC", oparam, option_mode=omode,
                                      source_shift0=ss)
        finally:
            A.plot_result_debug = orig
        out[f"af{k}_start"] = start
        out[f"af{k}_mode"] = np.array(oparam)
        out[f"af{k}_source_shift"] = np.array(ss, dtype=np.float64)
        out[f"af{k}_calls"] = np.array(log, dtype=np.float64)
        out[f"af{k}_params_after"] = live
        if oparam == "FoC":
            out[f"af{k}_detcenter"] = ret
        else:
            out[f"af{k}_ret"] = np.array([ret[0], ret[1]])
            assert ret[2] is live
        print("auto_focus_NA", name, len(log), "calls; params[0:2] ->", live[:2])

    out["meta_numpy"] = np.array(np.__version__)
    np.savez_compressed(os.path.join(MG.OUT, "akb_autofocus.npz"), **out)
    print("wrote", os.path.join(MG.OUT, "akb_autofocus.npz"))


if __name__ == "__main__":
    main()
