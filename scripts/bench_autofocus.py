"""Time the batched focus search on one MI355X:

    python scripts/bench_autofocus.py [--out gpurun_out/autofocus.json]

auto_focus_NA from the reference's best-alignment params (1800 'test' traces in the reference,
~17.5 s in the build container), its pieces (system build, one trace, one 100-plane sweep), a
batched trace of 256 systems, calc_FoC on a 5 x 5 source grid (25 FoC searches), the 'sep'
mode and auto_focus_sep ('abrr' and 'matrix'), and auto_focus_NA on KB_debug's pair (option_AKB
False: 1800 KB 'test' traces in the reference, 5.3 s on one core of the build container).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from akbraytracing_amd import autofocus as AF  # noqa: E402
from akbraytracing_amd import geometry as G  # noqa: E402


def best_params():
    p = np.zeros(26)
    p[0], p[1] = -5.73452570e-03, -2.87624337e-03
    p[8], p[9], p[13] = 1.05000000e-02, -3.59399021e-05, 2.39536993e-06
    p[20], p[21], p[25] = 1.05000000e-02, -3.59399021e-05, 2.39536993e-06
    return p


def wall(f, reps=1):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    p0 = best_params()
    res = {}
    # warm up: library load, kernels, rocm allocator
    AF.auto_focus_NA(50, p0.copy(), 1, 1, False, "", verbose=False)
    t, _ = wall(lambda: G.build_akb(p0), reps=20)
    res["build_ms"] = t * 1e3
    b = G.build_akb(p0)
    t, ts = wall(lambda: AF.TracedSystems([b]), reps=20)
    res["trace_one_system_ms"] = t * 1e3
    a = np.linspace(-0.3, 0.3, 100) + p0[0]
    t, _ = wall(lambda: ts.evaluate(a), reps=50)
    res["sweep_100_planes_ms"] = t * 1e3
    bs = [b] * 256
    t, _ = wall(lambda: AF.TracedSystems(bs, tilt=False), reps=5)
    res["trace_256_systems_ms"] = t * 1e3
    res["trace_256_systems_intersections_per_s"] = 256 * 53 * 53 * 4 / t

    calls = [0]

    class Counting(AF._SystemCache):
        def get(self, params, ss, tilt):
            ts = super().get(params, ss, tilt)
            outer = self

            class W:
                def evaluate(self_inner, a):
                    calls[0] += len(a)
                    return ts.evaluate(a)
            return W()

    t, ret = wall(lambda: AF.auto_focus_NA(50, p0.copy(), 1, 1, False, "", verbose=False,
                                           cache=Counting(True, 53)), reps=3)
    res["auto_focus_NA_ms"] = t * 1e3
    res["auto_focus_NA_test_traces_replaced"] = calls[0] // 3
    res["auto_focus_NA_reference_s"] = 17.46  # the reference, same call, build container (1 core)
    t, out = wall(lambda: AF.calc_FoC(p0.copy(), range_h=[-5e-3, 5e-3, 5], range_v=[-5e-3, 5e-3, 5]))
    res["calc_FoC_5x5_ms"] = t * 1e3
    # the 'sep' analysis (two-pass 53^2 trace, tilt, compare_sep's twenty searches in one launch)
    # and auto_focus_sep; the reference, same calls, build container (1 core): 2.0-2.3 s and 13.9 s
    from akbraytracing_amd import sep as S
    S.plot_result_sep(p0.copy(), verbose=False)
    t, _ = wall(lambda: S.plot_result_sep(p0.copy(), verbose=False), reps=5)
    res["sep_mode_ms"] = t * 1e3
    res["sep_mode_reference_s"] = 2.1
    t, _ = wall(lambda: S.auto_focus_sep(p0.copy(), 9, 21, -2e-5, 2e-5, option="abrr", verbose=False), reps=3)
    res["auto_focus_sep_abrr_ms"] = t * 1e3
    res["auto_focus_sep_abrr_reference_s"] = 13.9
    t, _ = wall(lambda: S.auto_focus_sep(p0.copy(), 9, 21, -2e-5, 2e-5, option="matrix", option_eval="9",
                                         verbose=False))
    res["auto_focus_sep_matrix_ms"] = t * 1e3
    # KB_debug's pair (option_AKB False)
    pk = np.zeros(26)
    pk[0], pk[1] = 2e-3, -1e-4
    AF.auto_focus_NA(50, pk.copy(), 1, 1, False, "", option_AKB=False, verbose=False)
    t, _ = wall(lambda: AF.kb_test(np.zeros(26)), reps=20)
    res["kb_test_mode_ms"] = t * 1e3
    res["kb_test_mode_reference_ms"] = 2.21
    t, _ = wall(lambda: AF.auto_focus_NA(50, pk.copy(), 1, 1, False, "", option_AKB=False, verbose=False), reps=3)
    res["kb_auto_focus_NA_ms"] = t * 1e3
    res["kb_auto_focus_NA_reference_s"] = 5.28
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
