"""The pruned PSF transform against rocFFT on the full plane for large pupils (512^2, 1024^2) at
several pad factors (psf_stack, HIP events, 5 repetitions):

    python scripts/micro_psf_large.py
"""
import os, sys, time, torch, numpy as np
sys.path.insert(0, os.getcwd())
from akbraytracing_amd import psf as G
res = {}
for n, pad in ((1024, 2), (1024, 4), (512, 2), (512, 4), (1024, 16)):
    o = torch.randn(n, n, dtype=torch.float64, device="cuda") * 1e-9
    for mode in ("fast", "rocfft"):
        if mode == "rocfft":
            os.environ["AKB_PSF_ROCFFT"] = "1"
        else:
            os.environ.pop("AKB_PSF_ROCFFT", None)
        ws = G.PsfWorkspace()
        G.psf_stack(o, None, [13.5e-9], 5e-6, pad_factor=pad, workspace=ws)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            G.psf_stack(o, None, [13.5e-9], 5e-6, pad_factor=pad, workspace=ws)
        b.record(); b.synchronize()
        res[(n, pad, mode)] = a.elapsed_time(b) / 5
    print(n, pad, {m: round(res[(n, pad, m)], 3) for m in ("fast", "rocfft")}, "ms", flush=True)
