"""The pipelined faithful PSF (akbraytracing_amd/faithful.py) against the host-synchronous drop-in
chain and against the reference's own PSF (MI355X).

Bars: the cone gridding is the global iteration's fixed-K result (bit for bit, test_gpu_parity);
against the converged chain (pupilmap.wave_pupil at scipy's tolerance + psfcalc.psf_calc) the maps
agree to 3e-7 of their range (the fixed sweep count's distance from the fixed point) and the PSF to
1e-7 of its peak; against the reference's PSF of its own run (akb_psf_full.npz) to the north star's
1e-6 of the peak.
"""
import numpy as np
import pytest
import torch

from conftest import golden, golden_json

pytestmark = pytest.mark.gpu


def _trace(n):
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    return RayWave(SystemGeometry.from_dict(golden_json("akb_geometry.json")), n).run()


def _crop(psf, fp, n):
    iy0, iy1, ix0, ix1 = (int(v) for v in fp[f"n{n}_psf_win"])
    return psf[iy0:iy1, ix0:ix1]


@pytest.mark.parametrize("n", [1001, pytest.param(3163, marks=pytest.mark.slow)])
def test_faithful_pipeline_vs_host_chain_and_reference(gpu, n):
    from akbraytracing_amd import pupilmap as PM
    from akbraytracing_amd.faithful import FaithfulPupil, image_axes_of
    from akbraytracing_amd.psfcalc import psf_calc
    out = _trace(n)
    d2 = out["detcenter2"]
    y, z, w2 = d2[1], d2[2], out["wave2"]
    fp_ = FaithfulPupil(n, n)
    r = fp_.run(y, z, w2)
    t = fp_.slots[0]["last"]
    t.check()
    torch.cuda.synchronize()
    # the host chain at scipy's tolerance
    m, gh, gv, _ = PM.wave_pupil(d2, w2, n, n, grid_num_H=128, grid_num_V=128)
    a = r["axes"].cpu().numpy()
    assert np.array_equal(a[:128], gh[0]) and np.array_equal(a[128:256], gv[:, 0])
    want_c = m.cpu().numpy()
    got_c = r["corrected"].cpu().numpy()
    rng_ = np.nanmax(want_c) - np.nanmin(want_c)
    assert np.array_equal(np.isnan(got_c), np.isnan(want_c))
    e_map = np.nanmax(np.abs(got_c - want_c)) / rng_
    GH, GV = gh - np.mean(gh), gv - np.mean(gv)
    host = psf_calc(m, GH, GV, 1e-2)
    P = r["psf"][0].cpu().numpy()
    e_psf = float(np.max(np.abs(P - host["psf"].cpu().numpy())))
    x_im, y_im = image_axes_of(r)
    assert np.array_equal(x_im, host["x_im"]) and np.array_equal(y_im, host["y_im"])
    fp = golden("akb_psf_full.npz")
    e_ref = float(np.max(np.abs(_crop(P, fp, n) - fp[f"n{n}_psf_crop"])))
    ch, est = r["change"].cpu().numpy().view(np.float64)
    print(f"n={n}: pipelined vs host chain: corrected map {e_map:.2e} of the range, PSF {e_psf:.2e} of the peak; "
          f"vs the reference's PSF {e_ref:.2e}; change at the target corners {ch:.2e}, value-error estimate "
          f"{est / rng_:.2e} of the range")
    assert est <= 1e-6 * rng_
    assert e_map <= 3e-7  # the cone solve's 12 sweeps against the host chain's converged gradients
    assert e_psf <= 1e-7
    assert e_ref <= 1e-6
    fp_.close()


def test_faithful_pipeline_in_flight_runs_equal_one_at_a_time(gpu):
    """Runs begun several at a time (tickets finished in order, pocket jobs on worker threads) give
    each run's own PSF bit for bit, as when each is begun and finished alone."""
    import copy
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    n = 401
    g = SystemGeometry.from_dict(golden_json("akb_geometry.json"))
    outs = []
    for i in range(4):
        gi = copy.deepcopy(g)
        gi.det2 = list(gi.det2[:3]) + [gi.det2[3] - 5e-6 * i]
        o = RayWave(gi, n).run()
        outs.append((o["detcenter2"][1].clone(), o["detcenter2"][2].clone(), o["wave2"].clone()))
    fp_ = FaithfulPupil(n, n, slots=3)
    alone = []
    for y, z, w in outs:
        alone.append(fp_.run(y, z, w)["psf"].clone())
    s = torch.cuda.Stream()
    tickets, got = [], []
    with torch.cuda.stream(s):
        for y, z, w in outs:
            tickets.append(fp_.begin(y, z, w, stream=s))
            if len(tickets) == 3:
                got.append(fp_.finish(tickets.pop(0), stream=s)["psf"].clone())
        while tickets:
            got.append(fp_.finish(tickets.pop(0), stream=s)["psf"].clone())
    torch.cuda.synchronize()
    for a, b in zip(alone, got):
        assert torch.equal(a, b)
    assert not torch.equal(alone[0], alone[3])
    fp_.close()


def test_faithful_pipeline_raises_for_a_missed_ray(gpu):
    from akbraytracing_amd.faithful import FaithfulPupil
    n = 65
    out = _trace(n)
    y = out["detcenter2"][1].clone()
    y[n * 10 + 5] = float("nan")
    fp_ = FaithfulPupil(n, n, slots=2)
    t = fp_.begin(y, out["detcenter2"][2], out["wave2"])
    with pytest.raises(ValueError):
        fp_.finish(t)
    fp_.close()


def _guard_case(geom, n, sweeps=None):
    """One run of geom at n^2 through FaithfulPupil: (its map and value-error estimate, the map from
    the converged gradients on the same axes, the map's range)."""
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.griddata import CubicGrid
    from akbraytracing_amd.wavefront import RayWave
    out = RayWave(geom, n).run()
    y, z, w = out["detcenter2"][1].contiguous(), out["detcenter2"][2].contiguous(), out["wave2"].contiguous()
    fp = FaithfulPupil(n, n, slots=2, **({"sweeps": sweeps} if sweeps else {}))
    t = fp.begin(y, z, w)
    r = fp.finish(t)
    got = r["map"].cpu().numpy().copy()
    est = float(r["change"].cpu().numpy().view(np.float64)[1])
    ax = r["axes"].cpu().numpy()
    cg = CubicGrid(y, z, n, n)
    ref = cg.interp(w.reshape(1, -1), ax[:128], ax[128:256], tol=1e-13).cpu().numpy()[0]
    rng_ = float(np.nanmax(ref) - np.nanmin(ref))
    return fp, t, got, est, ref, rng_, (y, z, w)


@pytest.mark.slow
def test_cone_guard_on_the_cycled_systems(gpu):
    """The cone solve's fixed CONE_SWEEPS against the converged gradients on every system the bench
    cycles (bench.system_variants of the C3 geometry), KB_debug's pair (configs[1]) and the C4 lattice
    (10000^2): each map within 3e-7 of its range of the converged one, the value-error estimate
    (the patches' corner bound, the band targets' value change of one more sweep) at least the
    map's actual error and inside the guard's bar, so Ticket.check() passes. With too few sweeps the guard trips and FaithfulPupil.run() returns the
    converged map instead."""
    import bench
    from akbraytracing_amd.griddata import CONE_GUARD, CONE_SWEEPS, ConeNotConverged
    from akbraytracing_amd.wavefront import SystemGeometry
    c3 = SystemGeometry.from_dict(golden_json("akb_geometry.json"))
    cases = [(f"c3 system {i}", g, 1001) for i, g in enumerate(bench.system_variants(c3, 8))]
    cases += [("c2 KB pair", SystemGeometry.from_dict(bench.geometry_dict("c2")), 1001), ("c4 lattice", c3, 10000)]
    for name, g, n in cases:
        fp, t, got, est, ref, rng_, _ = _guard_case(g, n)
        t.check()  # the guard passes at CONE_SWEEPS
        fp.close()
        assert np.array_equal(np.isnan(got), np.isnan(ref)), name
        err = float(np.nanmax(np.abs(got - ref)))
        print(f"{name} at {n}^2: {CONE_SWEEPS} sweeps vs converged {err / rng_:.2e} of the range, "
              f"estimate {est / rng_:.2e} (bar {CONE_GUARD:g})")
        assert err <= 3e-7 * rng_, name
        assert err <= est <= CONE_GUARD * rng_, name
    # too few sweeps: the estimate trips the guard; run() then forms the map from the converged gradients
    fp, t, got, est, ref, rng_, (y, z, w) = _guard_case(c3, 1001, sweeps=3)
    assert est > CONE_GUARD * rng_ and np.nanmax(np.abs(got - ref)) > 1e-6 * rng_
    with pytest.raises(ConeNotConverged):
        t.check()
    r = fp.run(y, z, w)
    assert r.get("converged") and np.nanmax(np.abs(r["map"].cpu().numpy() - ref)) <= 1e-6 * rng_
    fp.close()


# The moves the reference's alignment loops sweep (Legendrealignment calls, AKB_raytrace_20250312.py:
# 14664-14851; the loops themselves :13853-14043): params indices moved together, and the widest
# range each is swept over
ALIGN_MOVES = [((8, 20), 2e-3), ((10, 22), 1e-3), ((12, 24), 2e-3), ((9, 21), 1e-5), ((2, 14), 2e-5),
               ((2,), 1e-4), ((3,), 1e-5), ((4,), 1e-4), ((5,), 1e-6), ((7,), 1e-6), ((10,), 1e-5), ((11,), 1e-4),
               ((12,), 1e-5), ((14,), 1e-5), ((15,), 1e-5), ((16,), 1e-5), ((17,), 1e-5), ((19,), 1e-6),
               ((20,), 1e-4), ((21,), 1e-4), ((22,), 1e-4), ((23,), 1e-4), ((24,), 1e-5)]


@pytest.mark.slow
def test_cone_guard_on_drawn_misalignments(gpu):
    """the guard's value-error estimate bounds the actual error of the 12-sweep map
    (against the converged gradients on the same axes) on 50 systems drawn from the misalignments the
    reference's alignment loops sweep: each system 1-3 of ALIGN_MOVES, each uniform over its range,
    built by geometry.build_akb (the reference's plot_result_debug system) at 1001^2. A system the
    reference could not trace (np.inf) or whose lattice the device refuses is redrawn and counted."""
    from akbraytracing_amd import _lib
    from akbraytracing_amd import geometry as G
    from akbraytracing_amd.driver import ray_wave_conditions
    from akbraytracing_amd.griddata import CONE_GUARD
    from akbraytracing_amd.wavefront import SystemGeometry
    rng = np.random.default_rng(20260618)
    defocus_wave, _ = ray_wave_conditions(True)
    done, skipped, trips, ratios = 0, 0, 0, []
    while done < 50:
        assert skipped <= 50, "too many drawn systems refused"
        params = np.zeros(26)
        for k in rng.choice(len(ALIGN_MOVES), size=int(rng.integers(1, 4)), replace=False):
            idx, span = ALIGN_MOVES[k]
            params[list(idx)] += rng.uniform(-span, span)
        b = G.build_akb(params)
        if not isinstance(b, dict):
            skipped += 1
            continue
        det2 = np.zeros(10)
        det2[6] = 1
        det2[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]) + defocus_wave)
        geom = SystemGeometry.from_dict(dict(b, det2=[float(x) for x in det2], defocus_wave_m=defocus_wave))
        try:
            fp, t, got, est, ref, rng_, _ = _guard_case(geom, 1001)
        except (_lib.AKBError, ValueError):  # a ray missed, or a folded lattice: no pupil to grid
            skipped += 1
            continue
        fp.close()
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        err = float(np.nanmax(np.abs(got - ref)))
        assert err <= est, (params.tolist(), err, est)
        ratios.append(est / err if err > 0 else np.inf)
        trips += int(not (est <= CONE_GUARD * rng_))
        done += 1
    print(f"{done} drawn systems ({skipped} redrawn): estimate / actual error min {min(ratios):.2f}, "
          f"median {np.median(ratios):.2f}; guard trips {trips}")
