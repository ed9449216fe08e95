"""PSF timing alone on the GPU: pruned transform vs rocFFT on the full padded plane."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from akbraytracing_amd import psf as G

dev = torch.device("cuda")
rng = np.random.default_rng(0)
for (n, pad, lams) in ((128, 16, [13.5e-9]), (128, 16, [13.5e-9, 1.35e-9, 1.35e-10]), (256, 8, [13.5e-9]),
                       (1024, 2, [13.5e-9])):
    opd = torch.from_numpy(rng.standard_normal((n, n)) * 1e-9).to(dev)
    for mode in ("pruned", "rocfft"):
        if mode == "rocfft":
            os.environ["AKB_PSF_ROCFFT"] = "1"
        else:
            os.environ.pop("AKB_PSF_ROCFFT", None)
        ws = G.PsfWorkspace()
        out = None
        for _ in range(3):
            out = G.psf_stack(opd, None, lams, 5e-6, pad_factor=pad, workspace=ws, out=out)[0]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            G.psf_stack(opd, None, lams, 5e-6, pad_factor=pad, workspace=ws, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"{n}^2 pad {pad} x{len(lams)} {mode}: {ms * 1e3:.1f} us "
              f"({len(lams) * (n * pad) ** 2 * 8 / (ms * 1e-3) / 1e9:.0f} GB/s of f64 output)", flush=True)
