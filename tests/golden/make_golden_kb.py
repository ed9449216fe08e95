"""Record the reference's KB system construction and KB focus search (build container only; the
reference never travels to the GPU box):

    python tests/golden/make_golden_kb.py

KB_debug (AKB_raytrace_20250312.py:9742) builds its two-ellipse KB pair from KBdesign_7params
(:100) through KB_define (:297-336), aligns it on five centre rays and applies params'
misalignments (:10432-10934) before it traces; auto_focus_NA (:12746) with option_AKB = False
calls KB_debug(params, 1, 1, 'test') hundreds of times. Recorded per case, by wrapping the
reference's module-level primitives:

  k{k}_*   build cases: params, source_shift, designparams (or none) -> the two 53x53-ray quadrics
           in trace order, the detector plane's j, the 'test' return (vmirr_hyp, tilted hmirr_hyp,
           tilted detcenter, tilted angle).
  kaf_*    an auto_focus_NA run on the KB system: start params, the (params[0], params[1], std_v,
           std_h) of every 'test' call, the params after it and its return value.

Writes kb_build.npz (numpy 2.2, float64).
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


def cases():
    rng = np.random.default_rng(4242)
    scale = np.array([1e-3, 1e-4] + [1e-5, 1e-5, 1e-5, 1e-6, 1e-6, 1e-6] * 2 + [0.0] * 12)
    out = [(np.zeros(26), [0.0, 0.0, 0.0], None)]
    for _ in range(3):
        out.append((scale * rng.standard_normal(26), [0.0, 0.0, 0.0], None))
    p = np.zeros(26)
    p[2], p[8] = 2e-5, -1e-5  # pitches alone
    out.append((p, [0.0, 0.0, 0.0], None))
    out.append((scale * rng.standard_normal(26), [0.0, 1e-3, -2e-3], None))  # source shift
    out.append((np.zeros(26), [0.0, 0.0, 0.0], [146., 0.5, 0.25, 0.46, 0.082, 0.25, 0.14]))  # the paper design
    return out


def main():
    MG._stub_modules()
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_kb_"))
    import AKB_raytrace_20250312 as A
    out = {}
    for k, (p, ss, dp) in enumerate(cases()):
        rec = MG.Recorder(A)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                r = A.KB_debug(np.array(p, dtype=np.float64), 1, 1, "test", source_shift=list(ss), option_save=False,
                               designparams=None if dp is None else [np.float64(x) for x in dp])
        finally:
            rec.restore()
        big = MG.big(rec.calls, N53)
        isects = [c for c in big if c[0] == "mirr_ray_intersection"]
        planes = [c for c in big if c[0] == "plane_ray_intersection"]
        assert len(isects) == 2, len(isects)
        out[f"k{k}_params"] = np.array(p, dtype=np.float64)
        out[f"k{k}_source_shift"] = np.array(ss, dtype=np.float64)
        out[f"k{k}_design"] = np.array([] if dp is None else dp, dtype=np.float64)
        out[f"k{k}_coeffs"] = np.stack([c[1][0] for c in isects])
        out[f"k{k}_det_j"] = np.float64(planes[0][1][0][9])
        out[f"k{k}_dir0"] = isects[0][1][1]
        for name, v in zip(("vmirr_hyp", "hmirr_hyp", "detcenter", "angle"), r):
            out[f"k{k}_{name}"] = np.array(v)
        print("KB case", k, "std", np.std(r[2][2, :]), np.std(r[2][1, :]))

    A.option_AKB = False
    orig = A.KB_debug
    log = []

    def wrapped(params, na_h, na_v, option, *a, **kw):
        r = orig(params, na_h, na_v, option, *a, **kw)
        if option == "test":
            log.append((params[0], params[1], np.std(r[2][2, :]), np.std(r[2][1, :])))
        return r
    A.KB_debug = wrapped
    start = np.zeros(26)
    start[0], start[1] = 2e-3, -1e-4
    live = start.copy()
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            ret = A.auto_focus_NA(50, live, 1, 1, False, "")
    finally:
        A.KB_debug = orig
        A.option_AKB = True
    out["kaf_start"] = start
    out["kaf_calls"] = np.array(log, dtype=np.float64)
    out["kaf_params_after"] = live
    out["kaf_ret"] = np.array([ret[0], ret[1]])
    print("KB auto_focus_NA", len(log), "calls; params[0:2] ->", live[:2])
    out["meta_numpy"] = np.array(np.__version__)
    np.savez_compressed(os.path.join(MG.OUT, "kb_build.npz"), **out)
    print("wrote", os.path.join(MG.OUT, "kb_build.npz"))


if __name__ == "__main__":
    main()
