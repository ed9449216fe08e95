"""BASELINE configs[1]'s M1 -> M2 stage at its full size on one MI355X: KB_debug's pair traced on a
3163 x 3163 grid (saveWaveData, as tests/test_wavecalc_gpu.py builds it), the source -> M1 field on
all 1e7 M1 points, then M1 -> M2 over all 1e7 x 1e7 = 1e14 pairs (the driver's stage,
Wavecalc_raytrace_fromData_GPU0402_multi.py:466-474), in target chunks that each print a progress line
(each chunk passes the whole stage's source-split count, so every target's sum is the unchunked
call's bit for bit). Checks 24 sampled M2 targets against the oracle's C sum (<= 1e-9 of max |u|,
the Huygens bar) and writes one JSON record.

    python scripts/run_c2_m1m2_full.py [--n 3163] [--chunk 524288] [--out gpurun_out/c2_m1m2_full.json]
"""
import argparse
import hashlib
import json
import math
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=3163)
    p.add_argument("--chunk", type=int, default=1 << 19)
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c2_m1m2_full.json"))
    a = p.parse_args()
    import numpy as np
    import torch
    import oracle as O
    from akbraytracing_amd import wavedata as W
    from akbraytracing_amd.wavecalc import propagate, splits_for
    dev = torch.device("cuda", 0)
    k = 2 * np.pi / 13.5e-9
    with tempfile.TemporaryDirectory() as tmp:
        folder = W.saveWaveData(np.zeros(26), ray_num_H=a.n, directory=os.path.join(tmp, "w"), option_AKB=False,
                                defocus_for_wave=1e-3, downsample=(0, 0, 0, 0, 12, 12), timestamp="full")
        m1 = np.load(os.path.join(folder, "points_M1.npy"))
        m2 = np.load(os.path.join(folder, "points_M2.npy"))
        src = np.load(os.path.join(folder, "points_source.npy")).reshape(3, 1)
    n1, n2 = m1.shape[1], m2.shape[1]
    d = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)  # noqa: E731
    s1 = [d(m1[r]) for r in range(3)]
    u1 = propagate(*s1, *[d(src[r]) for r in range(3)], torch.ones(1, dtype=torch.complex128, device=dev), k)
    u1ds = u1 * d(m1[3])
    t2 = [d(m2[r]) for r in range(3)]
    sp = splits_for(n2, n1)
    out = torch.empty(n2, dtype=torch.complex128, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for c0 in range(0, n2, a.chunk):
        c1 = min(n2, c0 + a.chunk)
        out[c0:c1] = propagate(t2[0][c0:c1], t2[1][c0:c1], t2[2][c0:c1], *s1, u1ds, k, splits=sp)
        torch.cuda.synchronize()
        print(f"M1 -> M2: {c1} / {n2} targets, {time.perf_counter() - t0:.1f} s", flush=True)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    u2 = out.cpu().numpy()
    rng = np.random.default_rng(6)
    pick = np.sort(rng.choice(n2, 24, replace=False))
    want = O.huygens_c(m2[0, pick], m2[1, pick], m2[2, pick], m1[0], m1[1], m1[2], u1ds.cpu().numpy(), k)
    err = float(np.max(np.abs(u2[pick] - want)) / np.max(np.abs(want)))
    rec = {"stage": "configs[1] M1 -> M2 (Wavecalc_raytrace_fromData_GPU0402_multi.py:466-474), full size",
           "grid": a.n, "sources": int(n1), "targets": int(n2), "pairs": float(n1) * float(n2),
           "device_s": ms / 1e3, "pairs_per_s": float(n1) * float(n2) / (ms / 1e3), "chunks": math.ceil(n2 / a.chunk),
           "source_splits": sp, "finite": bool(np.all(np.isfinite(u2))),
           "sampled_targets_vs_oracle_max_rel_err": err, "bar": 1e-9, "ok": bool(err <= 1e-9 and np.all(np.isfinite(u2))),
           "sum_abs2": float(np.sum(np.abs(u2) ** 2)), "sha256_16": hashlib.sha256(u2.tobytes()).hexdigest()[:16]}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec), flush=True)
    return 0 if rec["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
