"""The N > 1 path on CPU: world_size 2 over gloo (127.0.0.1). Each rank traces its V-row shard
with the oracle's chain (the GPU kernels are covered by the gpu tests); the communicator must
reassemble exactly what one process sees."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle.pipeline as OPL
        from akbraytracing_amd.dist import TorchComm, split_counts
        from akbraytracing_amd.wavefront import Shard, sample_ownership, sample_plan
        with open(os.path.join(GOLDEN, "akb_geometry.json")) as f:
            g = json.load(f)
        comm = TorchComm()
        shard = Shard.split(n, world, rank)
        rand_h, rand_v, tan_h, tan_v = OPL.angle_tables(g, n)
        dirs = OPL.grid_dirs(tan_h, tan_v)
        lo, hi = shard.start, shard.start + shard.count
        _, r4, _ = OPL.chain(g["mirrors"], dirs[:, lo:hi].copy(), np.zeros((3, hi - lo)))
        # this rank's pieces of the resample picks, zero elsewhere (what RayWave._pass1 hands over)
        hb, he, col = sample_plan(n)
        sh = np.zeros(he - hb)
        sv = np.zeros(n)
        own_h, own_v = sample_ownership(shard, n)
        g_idx = np.arange(lo, hi)
        m = (g_idx >= hb) & (g_idx < he)
        sh[g_idx[m] - hb] = r4[1, m] / r4[0, m]
        cm = (g_idx % n) == col
        sv[g_idx[cm] // n] = r4[2, cm] / r4[0, cm]
        assert np.all(sh[~own_h] == 0) and np.all(sv[~own_v] == 0)
        sh, sv = comm.gather_samples(sh, sv, shard, n)
        # partial sums for the means: (sum, count) of this rank, summed across ranks
        part = torch.tensor([np.sum(r4[0]), float(r4.shape[1])], dtype=torch.float64)
        tot = comm.allreduce_sums(part).numpy()
        mx = comm.allreduce_max(torch.tensor([float(np.max(r4[1]))], dtype=torch.float64)).numpy()
        # Huygens-style field all-gather of uneven pieces
        counts = split_counts(10, world)
        piece = torch.arange(sum(counts[:rank]), sum(counts[:rank + 1]), dtype=torch.float64) * (1 + 1j)
        field = comm.allgather_field(piece.to(torch.complex128), counts).numpy()
        flags = comm.or_flags(1 | (rank << 3))  # rank 0: 0x1, rank 1: 0x9
        words = torch.tensor([1, rank << 30, -(1 << 31) if rank else 5], dtype=torch.int32)
        comm.allreduce_or(words)
        if rank == 0:
            np.savez(os.path.join(out_dir, "r0.npz"), sh=sh, sv=sv, tot=tot, mx=mx, field=field,
                     flags=np.array(flags), words=words.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [129, 181])  # shards hold whole 8192-ray buffers: >= 2 of them
def test_two_rank_shards_reassemble_single_process(tmp_path, n):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = np.load(os.path.join(tmp_path, "r0.npz"))
    import oracle.pipeline as OPL
    with open(os.path.join(GOLDEN, "akb_geometry.json")) as f:
        g = json.load(f)
    rand_h, rand_v, tan_h, tan_v = OPL.angle_tables(g, n)
    _, r4, _ = OPL.chain(g["mirrors"], OPL.grid_dirs(tan_h, tan_v), np.zeros((3, n * n)))
    _, v_idx, _, _, h_idx = OPL.sample_indices(n, n)
    assert np.array_equal(r["sh"], r4[1, h_idx] / r4[0, h_idx])
    assert np.array_equal(r["sv"], r4[2, v_idx] / r4[0, v_idx])
    # resample from the gathered picks equals the single-process resample exactly
    a = OPL.resample_from_angles(np.arctan(r["sh"]), np.arctan(r["sv"]), rand_h, rand_v)
    b = OPL.resample_tables(r4, rand_h, rand_v, n, n)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert r["tot"][1] == n * n
    assert abs(r["tot"][0] / r["tot"][1] - np.mean(r4[0])) < 1e-15
    assert r["mx"][0] == np.max(r4[1])
    assert np.array_equal(r["field"], np.arange(10) * (1 + 1j))
    # OR over ranks, not a sum: 0x1 | 0x9 = 0x9 (a sum would give 0xa, FLAG_ZERO_NORMAL | ...)
    assert int(r["flags"]) == 0x9
    assert r["words"].tolist() == [1, 1 << 30, -(1 << 31) | 5]


def _psf_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import akbraytracing_amd.psf as PSF
        from akbraytracing_amd.dist import TorchComm, psf_stack_sharded

        def fake_stack(opd, amp, lams, dx, pad_factor=2, **kw):
            # a stand-in transform (the kernel is a gpu test): plane b = opd tiled, times its wavelength
            t = opd.repeat(pad_factor, pad_factor)
            return torch.stack([t * lam for lam in lams]), None, None
        PSF.psf_stack = fake_stack
        opd = torch.arange(16, dtype=torch.float64).reshape(4, 4)
        lams = [13.5e-9, 1.35e-9, 1.35e-10]
        comm = TorchComm(torch.device("cpu"))
        mine_psf, mine = psf_stack_sharded(opd, lams, comm, pad_factor=2)
        full, order = psf_stack_sharded(opd, lams, comm, gather=True, pad_factor=2)
        np.savez(os.path.join(out_dir, f"psf{rank}.npz"), mine=np.array(mine),
                 mine_psf=mine_psf.numpy() if mine_psf is not None else np.zeros(0), full=full.numpy(),
                 order=np.array(order))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_wavelength_sharded_psf_stack(tmp_path, world):
    """the config-5 PSF stack, one wavelength per rank (lams[rank::world]); each
    wavelength transformed exactly once, and the gathered stack in wavelength order on every rank"""
    from akbraytracing_amd.dist import wavelength_shard
    lams = [13.5e-9, 1.35e-9, 1.35e-10]
    owned = sum((wavelength_shard(lams, world, r) for r in range(world)), [])
    assert sorted(owned) == sorted(lams) and wavelength_shard(lams, 1, 0) == lams
    mp.start_processes(_psf_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    want = np.stack([np.tile(np.arange(16.0).reshape(4, 4), (2, 2)) * lam for lam in lams])
    for r in range(world):
        d = np.load(os.path.join(tmp_path, f"psf{r}.npz"))
        assert d["mine"].tolist() == lams[r::world]
        assert np.array_equal(d["mine_psf"].reshape(-1), want[r::world].reshape(-1))
        assert np.array_equal(d["full"], want) and d["order"].tolist() == lams


def _huygens_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from akbraytracing_amd.dist import TorchComm, propagate_sharded

        def oracle_propagate(tx, ty, tz, sx, sy, sz, u, k):
            # the per-rank kernel's stand-in (the HIP kernel is a gpu test): the oracle's C sum
            return torch.from_numpy(O.huygens_c(tx.numpy(), ty.numpy(), tz.numpy(), sx.numpy(), sy.numpy(),
                                                sz.numpy(), u.numpy(), k))

        rng = np.random.default_rng(5)
        n, m = 101, 700  # 101 targets: uneven pieces over 2 and 3 ranks
        T = [torch.from_numpy(rng.random(n) * 1e-6 + o) for o in (1.0, 0.0, 0.0)]
        S = [torch.from_numpy(rng.random(m) * 1e-3) for _ in range(3)]
        u = torch.from_numpy(np.exp(2j * np.pi * rng.random(m)) * (1 + rng.random(m)))
        got = propagate_sharded(*T, *S, u, 2 * np.pi / 13.5e-9, TorchComm(), propagate=oracle_propagate)
        np.savez(os.path.join(out_dir, f"h{rank}.npz"), got=got.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_huygens_target_sharding_reassembles_one_process(tmp_path, world):
    """dist.propagate_sharded (the _multi script's target split, :123-229): targets
    in np.array_split pieces over the ranks, sources replicated, the field all-gathered in rank
    order on every rank - the one-process field, value for value (each target's sum is independent
    of the others; the HIP kernel's split order is pinned by tests/test_dist_gpu.py)."""
    import oracle as O
    mp.start_processes(_huygens_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rng = np.random.default_rng(5)
    n, m = 101, 700
    T = [rng.random(n) * 1e-6 + o for o in (1.0, 0.0, 0.0)]
    S = [rng.random(m) * 1e-3 for _ in range(3)]
    u = np.exp(2j * np.pi * rng.random(m)) * (1 + rng.random(m))
    want = O.huygens_c(*T, *S, u, 2 * np.pi / 13.5e-9)
    for r in range(world):
        assert np.array_equal(np.load(os.path.join(tmp_path, f"h{r}.npz"))["got"], want), r


def _gather_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from akbraytracing_amd.dist import TorchComm, gather_to_root
        counts = [5, 3, 4][:world]
        lo = sum(counts[:rank])
        a = torch.arange(lo, lo + counts[rank], dtype=torch.float64)
        c = a.to(torch.complex128) * (1 - 2j)
        got = gather_to_root(TorchComm(), [a, c], counts, root=1)
        np.savez(os.path.join(out_dir, f"g{rank}.npz"), none=np.array(got is None),
                 **({"a": got[0].numpy(), "c": got[1].numpy()} if got is not None else {}))
    finally:
        dist.destroy_process_group()


def test_gather_to_root_in_rank_order(tmp_path):
    """dist.gather_to_root (the faithful pupil's N > 1 route): uneven pieces, float and complex,
    concatenated in rank order on the root only."""
    world = 3
    mp.start_processes(_gather_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        d = np.load(os.path.join(tmp_path, f"g{r}.npz"))
        if r == 1:
            assert np.array_equal(d["a"], np.arange(12.0)) and np.array_equal(d["c"], np.arange(12.0) * (1 - 2j))
        else:
            assert bool(d["none"])
