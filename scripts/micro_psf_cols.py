"""The pruned PSF transform's kernels at the bench's size (128^2 pupil, pad 16 -> 2048^2) and the
example's (1024^2, pad 16 -> 16384^2): psf_stack on resident inputs, HIP events, ms per call and
GB/s of output (run under rocprofv3 --kernel-trace for the per-kernel split).

    python scripts/micro_psf_cols.py [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from akbraytracing_amd import psf as G
    for n, pad in ((128, 16), (1024, 16)):
        o = torch.randn(n, n, dtype=torch.float64, device="cuda") * 1e-9
        ws = G.PsfWorkspace()
        out = None
        for _ in range(2):
            out, _, _ = G.psf_stack(o, None, [13.5e-9], 5e-6, pad_factor=pad, workspace=ws, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = a.reps if n <= 256 else max(2, a.reps // 4)
        e0.record()
        for _ in range(reps):
            G.psf_stack(o, None, [13.5e-9], 5e-6, pad_factor=pad, workspace=ws, out=out)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"pupil": n, "pad": pad, "plane": n * pad, "ms": round(ms, 4),
                          "output_gbs": round((n * pad) ** 2 * 8 / (ms * 1e-3) / 1e9, 1)}), flush=True)
        del out, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
