"""The N > 1 path on the GPU: two ranks (gloo, both on cuda:0 - a rehearsal of the one-rank-per-GPU
RCCL run the driver makes on 8 GPUs) trace their buffer-aligned shards through the same pipeline
bench.py runs (pass 1 / resample / pass 2 on the main stream, tilt / OPD / pupil on a second
stream) and must reassemble what one process computes, bit for bit: every rank traces the same
pass-2 tables, and the means combine the ranks' numpy buffer sums in numpy's own order
(LeafSink.finish_dist)."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _geom():
    from akbraytracing_amd.wavefront import SystemGeometry
    return SystemGeometry.load(os.path.join(GOLDEN, "akb_geometry.json"))


def _systems(k):
    """k distinct systems (tests/test_gpu_parity.py::_variants): last mirror and detectors moved."""
    import copy
    from akbraytracing_amd.wavefront import SystemGeometry
    with open(os.path.join(GOLDEN, "akb_geometry.json")) as f:
        base = json.load(f)
    out = []
    for i in range(k):
        d = copy.deepcopy(base)
        d["mirrors"][-1]["coeffs"][9] = d["mirrors"][-1]["coeffs"][9] * (1.0 + 2e-11 * i)
        d["det1"][9] = d["det1"][9] - 3e-6 * i
        d["det2"][9] = d["det2"][9] - 5e-6 * i
        out.append(SystemGeometry.from_dict(d))
    return out


def _worker(rank, world, port, n, runs, out_dir, schedule="plain"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    from akbraytracing_amd.wavefront import RayWave, Shard
    AD.init_from_env()
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        rw = RayWave(_geom(), n, shard=Shard.split(n, world, rank), comm=AD.TorchComm(dev))
        bs = torch.cuda.Stream()
        outs = []

        def back(front):
            with torch.cuda.stream(bs):
                o = rw.launch_back(front, stream=bs)
                opd, _ = rw.pupil(32)
                outs.append({k: o[k].cpu().numpy() for k in ("last_hit", "wave2", "dist_err2")} |
                            {"pupil": opd.cpu().numpy()})

        if schedule == "plain":
            fronts = [rw.launch_front()]
            for _ in range(runs - 1):
                prev = fronts[-1]
                fronts.append(rw.launch_front(overlap=lambda p=prev: back(p)))
            back(fronts[-1])
        else:  # bench.py's --fuse 2 schedule, a different system per run
            sy = _systems(runs)
            nx = lambda i: sy[i + 1] if i + 1 < runs else None
            fr = []
            for i in range(runs):
                kw = dict(geometry=sy[i], next_geometry=nx(i))
                if len(fr) == 3:  # run i's pass 1 tilts run i-2 and forms run i-3's OPD
                    g = fr.pop(0)
                    fr.append(rw.launch_front(overlap=lambda p=g: back(p), fuse=fr[0], fuse_opd=g, **kw))
                else:
                    fr.append(rw.launch_front(fuse=fr[0] if len(fr) == 2 else None, **kw))
            for f in fr:
                back(f)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), start=rw.shard.start, count=rw.shard.count,
                 **{f"{k}_{i}": v for i, o in enumerate(outs) for k, v in o.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,schedule", [(129, "plain"), (129, "fuse2")])
def test_two_ranks_on_the_gpu_reassemble_one_process(gpu, tmp_path, n, schedule):
    """plain: the two-stream pipeline on one system; fuse2: bench.py's default schedule (run k's
    pass 1 tilts run k-2 and forms run k-3's OPD from cross-rank sums finished on their own stream),
    a different system per run, against one process's sequential run() of each system."""
    from akbraytracing_amd.wavefront import RayWave
    runs = 3 if schedule == "plain" else 6
    systems = [_geom()] * runs if schedule == "plain" else _systems(runs)
    rw = RayWave(_geom(), n)
    wants = []
    for g in systems:
        one = rw.run(geometry=g)
        wants.append(({k: one[k].cpu().numpy() for k in ("last_hit", "wave2", "dist_err2")},
                      rw.pupil(32)[0].cpu().numpy()))
    del rw, one
    torch.cuda.synchronize()
    mp.start_processes(_worker, args=(2, _free_port(), n, runs, str(tmp_path), schedule), nprocs=2, join=True,
                       start_method="spawn")
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(2)]
    for i in range(runs):
        want, want_pupil = wants[i]
        if schedule == "plain":  # (pipelined deeper, a run's pass-2 rows are rewritten by later runs')
            last_hit = np.concatenate([p[f"last_hit_{i}"] for p in parts], axis=1)
            assert np.array_equal(last_hit, want["last_hit"])  # pass 2: bit-exact per ray
        for k in ("wave2", "dist_err2"):  # the means in numpy's order across ranks: bit-exact too
            got = np.concatenate([p[f"{k}_{i}"] for p in parts])
            assert np.array_equal(got, want[k]), (i, k, np.max(np.abs(got - want[k])))
        for p in parts:  # every rank ends with the whole (all-reduced) pupil, OPD in metres
            assert np.array_equal(p[f"pupil_{i}"], want_pupil), i


def test_bench_two_ranks_runs_to_the_json_line(gpu, tmp_path):
    """bench.py under torchrun with two ranks (gloo on one GPU): every collective is reached by
    both ranks in the same order, so the run ends with rank 0's JSON line."""
    import subprocess
    import sys
    root = ROOT
    env = dict(os.environ, AKB_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--rays", "250000"]
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0


def test_bench_gpus_flag_launches_the_ranks(gpu):
    """`python bench.py --gpus 2` with no launcher starts its own two ranks (torch.distributed.run
    as a child, before anything touches the GPU): the line reports the world it ran, n_gpus == 2.
    gloo lets both ranks share the one GPU here; the driver's 8-GPU node runs RCCL."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["AKB_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rays", "1e5", "--steps", "2",
           "--warmup", "3", "--ramp-ms", "0", "--no-extras", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["value"] > 0
    assert out["config"]["rays_total"] == 447 * 447  # round(sqrt(2 x 1e5))^2: C4's weak-scaling grid


def _huygens_field(n, m, seed=3):
    rng = np.random.default_rng(seed)
    T = [rng.random(n) * 2e-6 + o for o in (1.0, 0.0, 0.0)]
    S = [rng.random(m) * 1e-3 for _ in range(3)]
    u = np.exp(2j * np.pi * rng.random(m)) * (1 + rng.random(m))
    return T, S, u


def _huygens_rank(rank, world, port, n, m, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    AD.init_from_env()
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        T, S, u = _huygens_field(n, m)
        td = [torch.from_numpy(a).to(dev) for a in T]
        sd = [torch.from_numpy(a).to(dev) for a in S]
        got = AD.propagate_sharded(*td, *sd, torch.from_numpy(u).to(dev), 2 * np.pi / 13.5e-9, AD.TorchComm(dev))
        np.savez(os.path.join(out_dir, f"h{rank}.npz"), got=got.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_huygens_sharded_over_ranks_is_one_process_bitwise(gpu, tmp_path, world):
    """dist.propagate_sharded through the HIP kernel (ranks over gloo on the one GPU): every rank
    sums its targets' sources in the whole problem's split order (wavecalc.splits_for), so the
    gathered field equals one process's propagate bit for bit - a split count > 1 here (4225
    targets cannot fill the chip alone)."""
    from akbraytracing_amd import wavecalc as W
    n, m = 4225, 300_000
    T, S, u = _huygens_field(n, m)
    assert W.splits_for(n, m) > 1
    want = W.propagate(*(torch.from_numpy(a).to(gpu) for a in T), *(torch.from_numpy(a).to(gpu) for a in S),
                       torch.from_numpy(u).to(gpu), 2 * np.pi / 13.5e-9).cpu().numpy()
    torch.cuda.synchronize()
    mp.start_processes(_huygens_rank, args=(world, _free_port(), n, m, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert np.array_equal(np.load(os.path.join(tmp_path, f"h{r}.npz"))["got"], want), r


def test_huygens_multi_gpu_threads_equal_one_device(gpu):
    """forward_propagation_cupy_batch_multi_gpu (the _multi script's thread per device, :123-229)
    with the device list [0, 0] (two host threads, one GPU): the concatenated pieces are the
    one-device field bit for bit, and the reference's dS scaling is applied on both paths."""
    from akbraytracing_amd import wavecalc as W
    n, m = 5001, 200_000
    T, S, u = _huygens_field(n, m, seed=9)
    ds = np.random.default_rng(1).random(m) * 1e-12 + 1e-12
    k = 2 * np.pi / 13.5e-9
    one = W.forward_propagation_numpy_batch(*T, *S, u, k, ds)
    two = W.forward_propagation_cupy_batch_multi_gpu(*T, *S, u, k, ds, devices=[0, 0])
    three = W.forward_propagation_cupy_batch_multi_gpu(*T, *S, u, k, ds, devices=[0, 0, 0])
    assert np.array_equal(two, one) and np.array_equal(three, one)


def _pupil_rank(rank, world, port, n, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    from akbraytracing_amd.wavefront import RayWave, Shard
    AD.init_from_env()
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        rw = RayWave(_geom(), n, shard=Shard.split(n, world, rank), comm=AD.TorchComm(dev))
        out = rw.run()
        got = AD.wave_pupil_sharded(rw, out, 64, AD.TorchComm(dev))
        if rank == 0:
            np.save(os.path.join(out_dir, "pupil.npy"), got[0].cpu().numpy())
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_faithful_pupil_gathered_from_eight_ranks(gpu, tmp_path):
    """SURVEY.md §8(e)'s route for the global griddata step: eight ranks (gloo, all on cuda:0) trace
    their shards of a 301 x 301 grid and hand their (y, z, Wave2) rows to rank 0, which grids the
    whole lattice - the one-process faithful pupil bit for bit (the sharded trace is bit-exact per
    ray, and the gather restores ray order)."""
    from akbraytracing_amd.pupilmap import wave_pupil
    from akbraytracing_amd.wavefront import RayWave
    n = 301
    out = RayWave(_geom(), n).run()
    want = wave_pupil(out["detcenter2"], out["wave2"], n, n, grid_num_H=64, grid_num_V=64)[0].cpu().numpy()
    torch.cuda.synchronize()
    mp.start_processes(_pupil_rank, args=(8, _free_port(), n, str(tmp_path)), nprocs=8, join=True,
                       start_method="spawn")
    assert np.array_equal(np.load(os.path.join(tmp_path, "pupil.npy")), want, equal_nan=True)
