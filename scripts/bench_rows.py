"""Measure the §8 rows beyond the traced step on one MI355X, each beside the CPU computation the
reference runs for it (the reference's own numpy / scipy calls, or the oracle's C restatement):

    python scripts/bench_rows.py [--n 3163] [--out profiles/r01c_rows.json]

Rows: f1 gridding chain (griddata x2 + nanmean + plane corrections), plane correction alone,
f2 find_defocus, f3 calc_dS, a13/f4 psf_calc, f4 match_legendre_multi. Device times are wall
times around the drop-in call with the device synchronised (they include the drop-ins' own host
steps and syncs); inputs are resident on the device first. CPU legs run on smaller inputs where
the reference would take minutes; sizes are in each record.
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


def dev_time(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def cpu_time(fn, reps=1):
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


def lattice(n, seed=0):
    u, v = np.meshgrid(np.linspace(-1, 1, n), np.linspace(-1, 1, n))
    X = u * 1e-4 + 3e-6 * v ** 2 - 2e-6 * u * v + 1e-6 * v ** 3
    Y = v * 1.3e-4 + 4e-6 * u ** 2 + 1e-6 * u ** 3
    rng = np.random.default_rng(seed)
    F = 0.3 * u ** 2 - 0.2 * u * v + 0.1 * np.sin(3 * v) + 1e-3 * rng.standard_normal(u.shape)
    return X, Y, F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3163)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from akbraytracing_amd import device as D
    from akbraytracing_amd import focus, psfcalc, pupilmap, wavedata
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    import oracle
    import oracle.pupilmap as OPM
    from scipy.interpolate import griddata as sp_griddata
    from scipy.ndimage import rotate as sp_rotate
    dev = D.device()
    n = a.n
    rows = []

    def emit(rec):
        rows.append(rec)
        print(json.dumps(rec), flush=True)

    # ---- f1: the gridding chain on an n x n lattice of hits (two value sets, as the driver)
    X, Y, F = lattice(n)
    det = torch.stack([torch.zeros(n * n, dtype=torch.float64), torch.from_numpy(X.ravel()),
                       torch.from_numpy(Y.ravel())]).to(dev)
    f = torch.from_numpy(F.ravel()).to(dev)
    t_dev = dev_time(lambda: pupilmap.wave_maps(det, f, 2 * f, n, n), reps=2)
    m = 401
    Xs, Ys, Fs = lattice(m)
    gx, gy = np.linspace(Xs.min(), Xs.max(), m), np.linspace(Ys.min(), Ys.max(), m)
    GH, GV = np.meshgrid(gx, gy)

    def cpu_f1():
        w = sp_griddata((Xs.ravel(), Ys.ravel()), Fs.ravel(), (GH, GV), method="cubic")
        d = sp_griddata((Xs.ravel(), Ys.ravel()), 2 * Fs.ravel(), (GH, GV), method="cubic")
        w = w - np.nanmean(w)
        OPM.plane_correction_with_nan_and_outlier_filter(w)
        OPM.plane_correction_with_nan_and_outlier_filter(d)
    t_cpu = cpu_time(cpu_f1)
    emit({"row": "f1 gridding chain (griddata cubic x2, nanmean, plane correction x2)", "device_points": n * n,
          "device_s": t_dev, "cpu_points": m * m, "cpu_s": t_cpu, "cpu": "scipy griddata + lstsq plane fits",
          "device_points_per_s": n * n / t_dev, "cpu_points_per_s": m * m / t_cpu})

    # ---- plane correction alone at n x n
    wmap = torch.from_numpy(F).to(dev)
    t_dev = dev_time(lambda: pupilmap.plane_correction_with_nan_and_outlier_filter(wmap))
    t_cpu = cpu_time(lambda: OPM.plane_correction_with_nan_and_outlier_filter(F))
    emit({"row": "f1 plane_correction_with_nan_and_outlier_filter", "points": n * n, "device_s": t_dev,
          "cpu_s": t_cpu, "cpu": "numpy lstsq restatement of the curve_fit pair", "speedup": t_cpu / t_dev})

    # ---- f2: find_defocus on the traced grid's exit rays (10 loops x 50 planes)
    geom = SystemGeometry.load(os.path.join(ROOT, "tests", "golden", "akb_geometry.json"))
    rw = RayWave(geom, n)
    out = rw.run(opd=False)
    s2f = -geom.det1[3]
    rays, pts = out["dir_out"], out["last_hit"]
    sweep = focus.PlaneSweep(rays, pts)
    t_dev = dev_time(lambda: focus.find_defocus(rays, pts, s2f, 0.0, n, sweep=sweep))
    k = 1001 * 1001
    r_np = rays[:, :k].cpu().numpy()
    p_np = pts[:, :k].cpu().numpy()

    def cpu_f2_loop():
        for j in np.linspace(-0.3, 0.3, 50):
            c = np.zeros(10)
            c[6] = 1
            c[9] = -(s2f + j)
            d = oracle.plane_ray_intersection(c, r_np, p_np)
            np.std(d[1, :])
            np.std(d[2, :])
    t_cpu = cpu_time(cpu_f2_loop) * 10  # 10 loops
    emit({"row": "f2 find_defocus (10 loops x 50 planes)", "device_rays": n * n, "device_s": t_dev,
          "cpu_rays": k, "cpu_s": t_cpu, "cpu": "oracle C plane_ray_intersection + np.std per plane",
          "device_ray_planes_per_s": n * n * 500 / t_dev, "cpu_ray_planes_per_s": k * 500 / t_cpu})
    del rw, out, sweep

    # ---- f3: calc_dS on the n x n hit grid
    pts3 = torch.stack([det[1], det[2], torch.from_numpy((X * Y).ravel()).to(dev)]).contiguous()
    t_dev = dev_time(lambda: wavedata.calc_dS(pts3, n, n))
    p_host = pts3.cpu().numpy()
    t_cpu = cpu_time(lambda: oracle.calc_dS(p_host, n, n))
    emit({"row": "f3 calc_dS", "points": n * n, "device_s": t_dev, "cpu_s": t_cpu,
          "cpu": "oracle C restatement (1 thread)", "device_gbs_algorithmic": n * n * 32 / t_dev / 1e9})

    # ---- a13 / f4: psf_calc on a measured-size map (65^2, the reference's run) and 257^2
    for size in (65, 257):
        u, v = np.meshgrid(np.linspace(-1, 1, size), np.linspace(-1, 1, size))
        mp_ = 0.02 * (u ** 2 - v ** 2) + 0.01 * u * v
        mp_[u ** 2 + v ** 2 > 0.95] = np.nan
        mp_[:3, :] = np.nan
        gh, gv = np.meshgrid(np.linspace(-5e-5, 5e-5, size), np.linspace(-5e-5, 5e-5, size))
        mdev = torch.from_numpy(mp_).to(dev)
        t_dev = dev_time(lambda: psfcalc.psf_calc(mdev, gh, gv, 0.01))
        pad = 16
        py = (size + size % 2) * pad

        def cpu_psf():
            filled = np.where(np.isnan(mp_), 0.0, mp_)
            r = sp_rotate(filled, 1.0, reshape=False, order=3)
            msk = sp_rotate((~np.isnan(mp_)).astype(float), 1.0, reshape=False, order=3)
            opd = np.where(msk < 0.5, 0.0, r / np.maximum(msk, 1e-12)) * 1e-9
            U = (msk >= 0.5) * np.exp(1j * 2 * np.pi / 13.5e-9 * opd)
            P = np.zeros((py, py), complex)
            P[:U.shape[0], :U.shape[1]] = U
            I = np.abs(np.fft.fftshift(np.fft.fft2(np.fft.ifftshift(P)))) ** 2
            return I / I.max()
        t_cpu = cpu_time(cpu_psf)
        emit({"row": f"a13 psf_calc {size}^2 (pad 16 -> {py}^2)", "device_s": t_dev, "cpu_s": t_cpu,
              "cpu": "scipy.ndimage.rotate order 3 x2 + numpy fft2 (the reference's calls)", "speedup": t_cpu / t_dev})

    # ---- f4: match_legendre_multi on an n x n map, order 5
    sq = torch.from_numpy(F).to(dev)
    t_dev = dev_time(lambda: pupilmap.match_legendre_multi(sq, 5))
    import oracle.legendre as OL
    m2 = 1001
    t_cpu = cpu_time(lambda: OL.fit_multi(F[:m2, :m2], 5))
    emit({"row": "f4 match_legendre_multi (order 5, 15 terms)", "device_points": n * n, "device_s": t_dev,
          "cpu_points": m2 * m2, "cpu_s": t_cpu, "cpu": "numpy restatement of legendre_fit",
          "device_points_per_s": n * n / t_dev, "cpu_points_per_s": m2 * m2 / t_cpu})

    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"n": n, "rows": rows, "host_threads": os.cpu_count()}, fh, indent=1)


if __name__ == "__main__":
    main()
