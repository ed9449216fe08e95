"""BASELINE configs at their own sizes against the oracle (MI355X).

C4 (configs[3]): the 10000^2 = 1e8-ray AKB ray_wave trace, 20000 sampled rays plus the resample picks
against oracle/pipeline.py: pass 2's hit on mirror 4, exit direction and OPL bit for bit (the oracle
traces the picks, resamples with numpy / scipy exactly as the driver does, then traces the sampled
rays), and - given the device's tilt matrices, centre and means, which only a full-grid reduction
forms - the tilted detector hits, DistError2 and Wave2 of the sampled rays bit for bit through the
oracle's own rotation and plane primitives.

C5 (configs[4]): the same at its own 10000^2 (1e8 rays) and at 3163^2 with the Legendre figure-error
OPL perturbation on every ray; the perturbation against oracle/legendre.py (to the OPL's rounding),
the rest as C4. And the config's three-wavelength PSF stack sharded one wavelength per rank
(dist.psf_stack_sharded, three gloo ranks on the one GPU, the real transform): each rank's plane and
the gathered stack equal the single-process stack bit for bit.

C2 (configs[1]): KB_debug's pair at params = 0 (bench.py --config c2's system) at its own 3163^2,
20000 sampled rays plus the picks against the oracle as C4.

AKB_raytrace_20250312.py:2694-2905 (grid, passes, resample), :3583-3677 (tilt, OPD), KB_debug
:10948-10997; legendre_fit.py:45-57; SURVEY.md §8(d).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O
import oracle.pipeline as OPL
from conftest import golden_json

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _sample(n, k, seed):
    _, v_idx, _, _, h_idx = OPL.sample_indices(n, n)
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([h_idx, v_idx, rng.integers(0, n * n, k), [0, n - 1, n * n - n, n * n - 1]]))


def _oracle_pass2(g, n, idx):
    """Pass 2 of the driver's trace on the rays idx: pass 1 of the resample's picks only, the
    equal-angle resample, then the chain on the sampled rays' directions."""
    rand_h, rand_v, tan_h, tan_v = OPL.angle_tables(g, n)
    col, v_idx, start, end, h_idx = OPL.sample_indices(n, n)
    src = np.zeros((3, 1))
    picks = np.concatenate([h_idx, v_idx])
    iv, ih = np.divmod(picks, n)
    d = O.normalize_vector(np.stack([np.ones(picks.size), tan_h[ih], tan_v[iv]]))
    _, r4, _ = OPL.chain(g["mirrors"], d, np.repeat(src, picks.size, axis=1))
    nh = h_idx.size  # resample_tables' arctans of the picks' exit slopes (:2857-2860)
    angle_h = np.arctan(r4[1, :nh] / r4[0, :nh])
    angle_v = np.arctan(r4[2, nh:] / r4[0, nh:])
    new_h, new_v = OPL.resample_from_angles(angle_h, angle_v, rand_h, rand_v)
    tan_h2 = np.tan(new_h)
    tan_v2 = np.array([np.tan(x) for x in new_v], dtype=np.float64)
    iv, ih = np.divmod(idx, n)
    d2 = O.normalize_vector(np.stack([np.ones(idx.size), tan_h2[ih], tan_v2[iv]]))
    hits, r4, segs = OPL.chain(g["mirrors"], d2, np.repeat(src, idx.size, axis=1), with_segments=True)
    opl = segs[0]
    for s in segs[1:]:
        opl = opl + s
    return hits[-1], r4, opl


def _oracle_rotate(ry, rz, centre, v):
    out = np.empty_like(v)
    c = None if centre is None else np.ascontiguousarray(centre, dtype=np.float64)
    O.lib().oracle_rotate(O._ptr(np.ascontiguousarray(ry)), O._ptr(np.ascontiguousarray(rz)),
                          None if c is None else O._ptr(c), O._ptr(np.ascontiguousarray(v)), v.shape[1], 1,
                          v.shape[1], O._ptr(out), v.shape[1])
    return out


def _oracle_opd(g, last_hit, dir_out, opl, params, means):
    """The tilt and OPD of the sampled rays (:3583-3677) with the device's rotation matrices / centre
    (params[2:23]) and the device's full-grid means (mean total 2, mean detector-1 focus)."""
    ry, rz, focus = params[2:11].reshape(3, 3), params[11:20].reshape(3, 3), params[20:23]
    d_rot = _oracle_rotate(ry, rz, None, dir_out)
    p_rot = _oracle_rotate(ry, rz, focus, last_hit)
    c2 = np.zeros(10)
    c2[6:10] = g["det2"][6:10]
    det2 = O.plane_ray_intersection(c2, d_rot, p_rot)
    total2 = opl + O.seglen(p_rot, det2)
    (mean_t1, mean_t2), mean_focus = means
    dist_err2 = (total2 - mean_t2) * 1e9
    sph = O.seglen(np.broadcast_to(np.asarray(mean_focus)[:, None], det2.shape).copy(), det2) * 1e9
    return det2, dist_err2, dist_err2 - sph


def _check_config(n, perturbation=None, k=20000, g=None):
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    g = golden_json("akb_geometry.json") if g is None else g
    rw = RayWave(SystemGeometry.from_dict(g), n, perturbation=perturbation)
    out = rw.run()
    torch.cuda.synchronize()
    assert out["flags"] == (0, 0)
    idx = _sample(n, k, n)
    ti = torch.from_numpy(idx).cuda()
    last_hit, dir_out, opl = _oracle_pass2(g, n, idx)
    assert np.array_equal(out["last_hit"][:, ti].cpu().numpy(), last_hit)
    assert np.array_equal(out["dir_out"][:, ti].cpu().numpy(), dir_out)
    got_opl = out["opl"][ti].cpu().numpy()
    if perturbation is None:
        assert np.array_equal(got_opl, opl)
    else:
        import oracle.legendre as OL
        want = OL.perturbation(n, n, perturbation.coeffs).reshape(-1)[idx]
        assert np.all(np.abs((got_opl - opl) - want) <= 1.01 * np.spacing(opl) + 1e-13 * np.abs(want))
        opl = got_opl  # the tilt / OPD below from the device's perturbed path length
    params = out.tilt_params()
    assert params is not None
    det2, e2, w2 = _oracle_opd(g, last_hit, dir_out, opl, params, rw.means())
    assert np.array_equal(out["detcenter2"][:, ti].cpu().numpy(), det2)
    assert np.array_equal(out["dist_err2"][ti].cpu().numpy(), e2)
    assert np.array_equal(out["wave2"][ti].cpu().numpy(), w2)
    return out


def test_c4_1e8_rays_sampled_vs_oracle(gpu):
    _check_config(10000)


@pytest.mark.parametrize("n", [3163, 10000])
def test_c5_perturbed_sampled_vs_oracle(gpu, n):
    """configs[4]: the Legendre-perturbed trace at 3163^2 and at the config's own 10000^2 (1e8 rays)."""
    from akbraytracing_amd.legendre import LegendrePerturbation, config5_coefficients
    pert = LegendrePerturbation(config5_coefficients())
    out = _check_config(n, perturbation=pert)
    assert bool(torch.isfinite(out["wave2"]).all())
    del out
    torch.cuda.empty_cache()


def test_c2_3163_kb_sampled_vs_oracle(gpu):
    """configs[1] at its own 3163^2: KB_debug's pair (bench.py --config c2), sampled rays bit for bit."""
    import bench
    out = _check_config(3163, g=bench.geometry_dict("c2"))
    assert bool(torch.isfinite(out["wave2"]).all())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stack_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    AD.init_from_env()
    try:
        dev = torch.device("cuda", 0)
        opd = torch.from_numpy(np.load(os.path.join(out_dir, "opd.npy"))).to(dev)
        lams = [13.5e-9, 1.35e-9, 1.35e-10]
        comm = AD.TorchComm(dev)
        mine, held = AD.psf_stack_sharded(opd, lams, comm, pad_factor=16)
        full, order = AD.psf_stack_sharded(opd, lams, comm, gather=True, pad_factor=16)
        np.savez(os.path.join(out_dir, f"stack{rank}.npz"), held=np.array(held),
                 mine=mine.cpu().numpy() if mine is not None else np.zeros(0), full=full.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_c5_wavelength_sharded_psf_stack_real_kernel(gpu, tmp_path):
    """Config 5's three-wavelength stack of a real 128^2 pupil (the C3 trace's faithful pupil) over
    three gloo ranks sharing the GPU: rank r transforms lams[r] with the device kernel; its plane and
    the all-gathered stack equal the single-process stack_psf of all three, bit for bit."""
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.psf import psf_stack
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    n = 1001
    out = RayWave(SystemGeometry.from_dict(golden_json("akb_geometry.json")), n).run()
    fp = FaithfulPupil(n, n, slots=2)
    r = fp.run(out["detcenter2"][1], out["detcenter2"][2], out["wave2"])
    opd = r["rotated"] * 1e-9
    fp.close()
    np.save(os.path.join(tmp_path, "opd.npy"), opd.cpu().numpy())
    lams = [13.5e-9, 1.35e-9, 1.35e-10]
    want = psf_stack(opd, None, lams, None, pad_factor=16)[0].cpu().numpy()
    torch.cuda.synchronize()
    world = 3
    mp.start_processes(_stack_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for rk in range(world):
        d = np.load(os.path.join(tmp_path, f"stack{rk}.npz"))
        assert d["held"].tolist() == lams[rk::world]
        assert np.array_equal(d["mine"].reshape(want[rk::world].shape), want[rk::world])
        assert np.array_equal(d["full"], want)
