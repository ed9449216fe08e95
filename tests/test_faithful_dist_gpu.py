"""The sharded faithful pupil (akbraytracing_amd/faithful_dist.py) against the one-process
FaithfulPupil, bit for bit: gloo ranks sharing the one GPU, each tracing its Shard.split rows with
RayWave and handing only its halo rows and its part of the boundary band on; the band owner's map,
corrected / rotated pupil, plane parameters and PSF must equal the unsharded chain's. Two runs
through two slots (the pipelined form), then a third with one non-finite hit on the last rank:
every rank completes the collectives and the band owner raises the one-process ValueError.
AKB_raytrace_20250312.py:3653-3716 (griddata -> nanmean -> plane correction -> psf_calc).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN

pytestmark = [pytest.mark.gpu]

KEYS = ("map", "corrected", "rotated", "params", "psf")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _geom():
    from akbraytracing_amd.wavefront import SystemGeometry
    return SystemGeometry.load(os.path.join(GOLDEN, "akb_geometry.json"))


def save_result(path, res):
    np.savez(path, **{k: res[k].cpu().numpy() for k in KEYS})


def assert_same(path, want):
    got = np.load(path)
    for k in KEYS:
        w = want[k].cpu().numpy() if isinstance(want[k], torch.Tensor) else want[k]
        assert np.array_equal(got[k], w, equal_nan=True), k


def sharded_worker(rank, world, port, n, out_dir, size=128, nan_run=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    from akbraytracing_amd.faithful_dist import ShardedFaithfulPupil
    from akbraytracing_amd.wavefront import RayWave, Shard
    AD.init_from_env()
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        comm = AD.TorchComm(dev)
        rw = RayWave(_geom(), n, shard=Shard.split(n, world, rank), comm=comm)
        out = rw.run()
        d2, w2 = out["detcenter2"], out["wave2"]
        sp = ShardedFaithfulPupil(n, comm, size=size, slots=2)
        t1 = sp.begin(d2[1], d2[2], w2)
        t2 = sp.begin(d2[1], d2[2], w2)
        r1 = sp.finish(t1)
        sp.check(t1)
        if rank == 0:
            save_result(os.path.join(out_dir, "run1.npz"), r1)
        r2 = sp.finish(t2)
        sp.check(t2)
        if rank == 0:
            save_result(os.path.join(out_dir, "run2.npz"), r2)
        else:
            assert r1 is None and r2 is None
        raised = "none"
        if nan_run:
            y = d2[1].clone()
            if rank == world - 1:
                y[y.shape[0] // 2] = float("nan")
            t3 = sp.begin(y, d2[2], w2)
            sp.finish(t3)
            try:
                sp.check(t3)
            except ValueError as e:
                raised = str(e)
        with open(os.path.join(out_dir, f"raised{rank}.txt"), "w") as f:
            f.write(raised)
        sp.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(1001, 3), (301, 8)])
def test_sharded_faithful_pupil_equals_one_process(gpu, tmp_path, n, world):
    """1001^2 over 3 ranks (~334 rows each), and 301^2 over 8 (~38 rows each: every window reaches
    into the band and past its neighbours)."""
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.wavefront import RayWave
    out = RayWave(_geom(), n).run()
    fp = FaithfulPupil(n, n, slots=2)
    want = fp.run(out["detcenter2"][1], out["detcenter2"][2], out["wave2"])
    want = {k: want[k].clone() for k in KEYS}
    torch.cuda.synchronize()
    fp.close()
    mp.start_processes(sharded_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    assert_same(os.path.join(tmp_path, "run1.npz"), want)
    assert_same(os.path.join(tmp_path, "run2.npz"), want)
    raised = [open(os.path.join(tmp_path, f"raised{r}.txt")).read() for r in range(world)]
    assert "non-finite" in raised[0]
    assert all(r == "none" for r in raised[1:])


def guard_worker(rank, world, port, n, out_dir, sweeps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    from akbraytracing_amd.faithful_dist import ShardedFaithfulPupil
    from akbraytracing_amd.wavefront import RayWave, Shard
    AD.init_from_env()
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        comm = AD.TorchComm(dev)
        rw = RayWave(_geom(), n, shard=Shard.split(n, world, rank), comm=comm)
        out = rw.run()
        d2, w2 = out["detcenter2"], out["wave2"]
        sp = ShardedFaithfulPupil(n, comm, size=128, slots=2, sweeps=sweeps)
        r, _ = sp.run(d2[1], d2[2], w2)  # every rank returns: the guard's verdict is broadcast
        if rank == 0:
            assert r.get("converged")
            save_result(os.path.join(out_dir, "guard.npz"), r)
        else:
            assert r is None
        r2, _ = sp.run(d2[1], d2[2], w2)  # and the group is still in step for the next run
        if rank == 0:
            save_result(os.path.join(out_dir, "guard2.npz"), r2)
        with open(os.path.join(out_dir, f"guard{rank}.txt"), "w") as f:
            f.write("ok")
        sp.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_cone_guard_trip_falls_back_on_every_rank(gpu, tmp_path):
    """A cone solve of 3 sweeps trips the guard on the band owner: the verdict is
    broadcast, the ranks' hits meet on the band owner, which forms the map from the converged
    gradients - FaithfulPupil.run's fallback, bit for bit - and every rank returns normally and
    runs the next run's collectives."""
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.wavefront import RayWave
    n, world = 1001, 3
    out = RayWave(_geom(), n).run()
    fp = FaithfulPupil(n, n, slots=2, sweeps=3)
    want = fp.run(out["detcenter2"][1], out["detcenter2"][2], out["wave2"])
    assert want.get("converged")
    want = {k: want[k].clone() for k in KEYS}
    torch.cuda.synchronize()
    fp.close()
    mp.start_processes(guard_worker, args=(world, _free_port(), n, str(tmp_path), 3), nprocs=world, join=True,
                       start_method="spawn")
    assert all(open(os.path.join(tmp_path, f"guard{r}.txt")).read() == "ok" for r in range(world))
    assert_same(os.path.join(tmp_path, "guard.npz"), want)
    assert_same(os.path.join(tmp_path, "guard2.npz"), want)
