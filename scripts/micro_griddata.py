"""Per-stage device timings of the griddata pieces on an n x n lattice (HIP events), for A/B of
the AKB_GD_* knobs: python scripts/micro_griddata.py [--n 3163]."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_griddata import lattice  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3163)
    ap.add_argument("--sweeps", type=int, default=16)
    a = ap.parse_args()
    from akbraytracing_amd import _lib, device as D
    from akbraytracing_amd.griddata import CubicGrid
    L = _lib.lib()
    X, Y, F = lattice(a.n)
    dev = D.device()
    cg = CubicGrid(torch.from_numpy(X.ravel()).to(dev), torch.from_numpy(Y.ravel()).to(dev), a.n, a.n)
    f = torch.from_numpy(np.stack([F.ravel(), 2 * F.ravel()])).to(dev)
    n = a.n * a.n
    g = [torch.zeros((2, n, 2), dtype=D.F64, device=dev) for _ in range(2)]
    chg = torch.zeros(a.sweeps + 1, dtype=torch.int64, device=dev)
    ring = torch.empty(10 * cg.L, dtype=D.F64, device=dev)
    s = D.stream_handle()
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("AKB_GD")}}
    for nv in (2, 1):
        for rep in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(a.sweeps):
                _lib.check(L.akb_gd_grad_sweep_f64(*cg._tri_args(), D.ptr(cg.xptr), D.ptr(cg.xidx), D.ptr(f), nv,
                                                   D.ptr(g[k & 1]), D.ptr(g[1 - (k & 1)]), D.ptr(ring), D.ptr(chg[k:]), s))
            e1.record()
            torch.cuda.synchronize()
        res[f"sweep_ms_nv{nv}"] = e0.elapsed_time(e1) / a.sweeps
    gx = torch.from_numpy(np.linspace(X.min(), X.max(), a.n)).to(dev)
    gy = torch.from_numpy(np.linspace(Y.min(), Y.max(), a.n)).to(dev)
    owner = torch.empty(n, dtype=torch.int32, device=dev)
    out = torch.empty((2, n), dtype=D.F64, device=dev)
    for rep in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(L.akb_gd_eval_f64(*cg._tri_args(), D.ptr(gx), a.n, D.ptr(gy), a.n, D.ptr(f), D.ptr(g[0]), 2,
                                     D.ptr(owner), D.ptr(out), s))
        e1.record()
        torch.cuda.synchronize()
    res["claim_eval_ms"] = e0.elapsed_time(e1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
