"""The sharded faithful pupil's plan and data movement on CPU (akbraytracing_amd/faithful_dist.py).

ShardPlan: every rank's window backs every vertex its cone patches, claims and cell pass read
(the patch box of an interior cell is rows iv - K - 1 .. iv + K + 2, akb_griddata.hip
k_gd_cone_assign / k_gd_cone_patch); the halo runs tile the window outside the rank's own rays, each
from the rank that owns them, and sends mirror receives; the band runs of all ranks are exactly the
vertices / cells of depth <= 2K + 3 (what the band iteration of depth 2K + 2 reads). Then the data
movement with gloo on CPU tensors at world 2 and 3: each rank's window equals the global lattice's
rows, and the band owner's full buffers equal the global lattice on the band.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from akbraytracing_amd.faithful_dist import ShardPlan, band_depth

K = 14


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _runs_to_set(runs):
    return set(np.concatenate([np.arange(a, b) for a, b in runs]).tolist()) if runs else set()


def _check_plan(n, world):
    plans = [ShardPlan.make(n, world, r, K) for r in range(world)]
    own = [p.own for p in plans]
    assert own[0][0] == 0 and own[-1][1] == n * n
    assert all(own[i][1] == own[i + 1][0] for i in range(world - 1))
    # claim windows cover every cell row; each holds every cell whose first corner is in my rays
    covered = set()
    for p in plans:
        r0, r1 = p.claim
        covered |= set(range(r0, r1))
        first, last = p.own[0] // n, min((p.own[1] - 1) // n, n - 2)
        assert r0 <= first and last < r1
    assert covered == set(range(n - 1))
    for p in plans:
        R0, R1 = p.rows
        c0, c1 = p.cells
        # the cell pass reads its cells' corners and the next row's cell (top edge)
        assert R0 <= c0 and (c1 + 1 <= R1 - 1 or c1 == n - 1)
        assert p.claim[0] >= R0 and p.claim[1] + 1 <= R1  # claimed cells' corners
        # interior targets whose cell's first corner is mine: the patch box in the window
        for iv in range(p.own[0] // n, min((p.own[1] - 1) // n, n - 2) + 1):
            if iv - K - 1 >= 1 and iv + K + 2 <= n - 2:
                assert R0 <= iv - K - 1 and iv + K + 2 < R1
                assert c0 <= iv - K - 1 and iv + K + 1 < c1
        # buffers: the band owner's are full size
        if p.is_root:
            assert p.base == 0 and p.nrows == n
        else:
            assert p.base == R0 and p.nrows == R1 - R0
        # halo receives tile the window outside my rays, each run inside its sender's rays
        window = set(range(R0 * n, R1 * n)) if n <= 400 else None
        got = set()
        for j, a, b in p.halo_recv:
            assert plans[j].own[0] <= a < b <= plans[j].own[1]
            assert (p.rank, a, b) in plans[j].halo_send
            if window is not None:
                got |= set(range(a, b))
        for i, a, b in p.halo_send:
            assert (p.rank, a, b) in plans[i].halo_recv
        if window is not None:
            mine = set(range(*p.own)) & window
            assert got | mine == window and not (got & mine)
    # the band: exactly the vertices / cells of depth <= 2K + 3, split by owner
    d = band_depth(K) + 1
    iv, ih = np.divmod(np.arange(n * n), n)
    depth_v = np.minimum(np.minimum(iv, ih), np.minimum(n - 1 - iv, n - 1 - ih))
    want_v = set(np.nonzero(depth_v <= d)[0].tolist())
    cv, ch = np.divmod(np.arange((n - 1) * (n - 1)), n - 1)
    depth_c = np.minimum(np.minimum(cv, ch), np.minimum(n - 2 - cv, n - 2 - ch))
    want_c = set(np.nonzero(depth_c <= d)[0].tolist())
    all_v, all_c = set(), set()
    p0 = plans[0]
    for r in range(world):
        sv, sc = _runs_to_set(p0.band_v[r]), _runs_to_set(p0.band_c[r])
        assert not (all_v & sv) and not (all_c & sc)
        assert all(own[r][0] <= v < own[r][1] for v in sv)
        all_v |= sv
        all_c |= sc
    assert all_v == want_v and all_c == want_c


@pytest.mark.parametrize("n,world", [(129, 2), (301, 2), (301, 3), (301, 8), (317, 3), (1001, 4)])
def test_shard_plan_covers_what_the_kernels_read(n, world):
    _check_plan(n, world)


def test_shard_plan_c4_eight_ranks():
    """configs[3]: 10000^2 over 8 ranks - windows of ~1290 rows, the halo from the two neighbours
    only, the band 1.2e6 vertices (29 MB of (y, z, Wave2)) instead of 1e8."""
    n, world = 10000, 8
    plans = [ShardPlan.make(n, world, r, K) for r in range(world)]
    for p in plans:
        assert {j for j, _, _ in p.halo_recv} <= {p.rank - 1, p.rank + 1}
        assert p.rows[1] - p.rows[0] <= n // world + 2 * (K + 3) + 3
    band = sum(plans[0].band_count(r) for r in range(world))
    d = band_depth(K) + 1
    assert band == n * n - (n - 2 * (d + 1)) ** 2
    assert band * 24 < 32e6


def _lattice(n):
    """A synthetic (y, z, f) lattice and diagonal pattern, the same on every rank."""
    i = torch.arange(n * n, dtype=torch.float64)
    vals = torch.stack([i * 0.5 + 1, -i * 0.25, torch.sin(i)])
    diag = (torch.arange((n - 1) * (n - 1)) * 7 % 3 == 0).to(torch.uint8)
    return vals, diag


def _move_worker(rank, world, port, n, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from akbraytracing_amd.dist import TorchComm
        from akbraytracing_amd.faithful_dist import BandGather, exchange_halo
        comm = TorchComm()
        p = ShardPlan.make(n, world, rank, K)
        vals, diag_g = _lattice(n)
        win = torch.full((3, p.nrows * n), float("nan"), dtype=torch.float64)
        exchange_halo(p, comm, vals[:, p.own[0]:p.own[1]].clone(), win)
        off = p.base * n
        R0, R1 = p.rows
        ok_win = bool(torch.equal(win[:, R0 * n - off:R1 * n - off], vals[:, R0 * n:R1 * n]))
        # the cell pass's diagonals over my cell rows (from the global pattern)
        diag = torch.full((max(p.nrows - 1, 1) * (n - 1),), 255, dtype=torch.uint8)
        c0, c1 = p.cells
        coff = p.base * (n - 1)
        diag[c0 * (n - 1) - coff:c1 * (n - 1) - coff] = diag_g[c0 * (n - 1):c1 * (n - 1)]
        BandGather(p, torch.device("cpu"))(comm, win, diag)
        res = dict(ok_win=ok_win)
        if p.is_root:
            d = band_depth(K) + 1
            iv, ih = np.divmod(np.arange(n * n), n)
            band = np.minimum(np.minimum(iv, ih), np.minimum(n - 1 - iv, n - 1 - ih)) <= d
            bi = torch.from_numpy(np.nonzero(band)[0])
            res["ok_band"] = bool(torch.equal(win[:, bi], vals[:, bi]))
            cv, ch = np.divmod(np.arange((n - 1) * (n - 1)), n - 1)
            cb = np.minimum(np.minimum(cv, ch), np.minimum(n - 2 - cv, n - 2 - ch)) <= d
            ci = torch.from_numpy(np.nonzero(cb)[0])
            res["ok_cells"] = bool(torch.equal(diag[ci], diag_g[ci]))
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array([int(v) for v in res.values()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(301, 2), (301, 3)])
def test_halo_and_band_movement_gloo(tmp_path, n, world):
    mp.start_processes(_move_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        got = np.load(os.path.join(tmp_path, f"r{r}.npy"))
        assert got.all(), (r, got)
        assert got.size == (3 if r == 0 else 1)


def test_pack_pockets_prefix():
    """faithful.pack_pockets: the device's pocket arrays packed into one prefix of the block
    (tri | nbr | edge | xptr | xidx[:xptr[L]]), the H2D copy's extent; the empty block too."""
    from akbraytracing_amd.faithful import pack_pockets
    rng = np.random.default_rng(3)
    for Lr, npk in ((10, 4), (37, 0), (64, 50)):
        cap = Lr
        o = dict(tri=0, nbr=3 * cap, edge=6 * cap, xptr=6 * cap + Lr, xidx=6 * cap + 2 * Lr + 1)
        o["npk"] = o["xidx"] + 6 * cap
        buf = rng.integers(-5, 1000, o["npk"] + 1).astype(np.int32)
        buf[o["npk"]] = npk
        xp = np.concatenate([[0], np.cumsum(rng.integers(0, 3, Lr))]) if npk else np.zeros(Lr + 1, np.int64)
        buf[o["xptr"]:o["xptr"] + Lr + 1] = xp
        want = {k: buf[o[k]:o[k] + c].copy() for k, c in
                (("tri", 3 * npk), ("nbr", 3 * npk), ("edge", Lr), ("xptr", Lr + 1), ("xidx", int(xp[-1])))}
        n, p = pack_pockets(buf, o, Lr)
        assert n == npk and p["len"] == 6 * npk + 2 * Lr + 1 + int(xp[-1])
        for k, w in want.items():
            assert np.array_equal(buf[p[k]:p[k] + w.size], w), k
