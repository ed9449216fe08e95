"""psf_fft_example.py's transform (1024^2 pupil, pad_factor=16 -> 16384^2) on one MI355X:

    python scripts/bench_psf_example.py [--out gpurun_out/psf_example.json]

Times the drop-in call (host arrays in, a 2 GiB numpy PSF out) and the device part alone
(psf_stack on resident inputs, HIP events), against the reference's numpy run recorded with the
fixture (tests/golden/psf_example.npz: reference_seconds).
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
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from akbraytracing_amd import psf as PSF  # noqa: E402
from make_golden_psf_example import example_inputs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    opd, amp, wl, dx, f = example_inputs()
    res = {"pupil": list(opd.shape), "pad_factor": 16, "output": [16384, 16384]}
    PSF.compute_psf_fft(opd, amp, wl, dx, f, pad_factor=16)  # warm-up: plans, workspace
    torch.cuda.synchronize()
    t = time.perf_counter()
    psf, x_im, y_im = PSF.compute_psf_fft(opd, amp, wl, dx, f, pad_factor=16)
    res["dropin_call_s"] = time.perf_counter() - t
    del psf
    o = torch.from_numpy(opd).cuda()
    a = torch.from_numpy(amp).cuda()
    out = torch.empty((1, 16384, 16384), dtype=torch.float64, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    PSF.psf_stack(o, a, [wl], dx, dx, pad_factor=16, out=out)
    e0.record()
    for _ in range(reps):
        PSF.psf_stack(o, a, [wl], dx, dx, pad_factor=16, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res["device_ms"] = ms
    res["output_gbs"] = 16384 * 16384 * 8 / (ms * 1e-3) / 1e9
    ref = np.load(os.path.join(ROOT, "tests", "golden", "psf_example.npz"))
    res["reference_numpy_s"] = float(ref["reference_seconds"])
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
