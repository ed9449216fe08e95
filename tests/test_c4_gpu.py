"""BASELINE configs[3] ("C4") on one MI355X: the 10000 x 10000 (1e8-ray) AKB ray_wave trace, once
unsharded and once as the 8-rank run the driver makes on 8 GPUs - eight processes (gloo, all on
cuda:0), each tracing its shard (Shard.split: 1525-1526 whole 8192-ray buffers, ~1250 V-rows) and
combining the means through the communicator. Everything must come out bit-exact: pass 2 (every
rank traces the same pass-2 tables), and Wave2 after the tilt, whose means combine the ranks'
numpy buffer sums in numpy's order (LeafSink.finish_dist); the trace flags clean.
Then the faithful pupil and PSF (griddata cubic -> nanmean -> plane correction -> psf_calc) of the
1e8 hits on one GPU (faithful.FaithfulPupil), and sharded over the eight ranks without gathering the
hits (faithful_dist.ShardedFaithfulPupil: halo rows to the neighbours, the boundary band to rank
0): the same map, pupil and PSF bit for bit.
AKB_raytrace_20250312.py:2694-2717 (the grid), :3653-3696 (the gridding), SURVEY.md §8(d) C4."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N = 10000
WORLD = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _geom():
    from akbraytracing_amd.wavefront import SystemGeometry
    return SystemGeometry.load(os.path.join(GOLDEN, "akb_geometry.json"))


BLOCK = 8192


def block_checksums(out):
    """One int64 per 8192-ray block of this shard (shards start at block boundaries) over the bits
    of pass 2's last hit, exit direction and OPL and of Wave2 (odd position weights, wrapping
    arithmetic): equal checksums <=> equal bits, barring a 2^-64 collision."""
    m = out["opl"].shape[0]
    pad = (-m) % BLOCK
    rows = [out["last_hit"], out["dir_out"], out["opl"].unsqueeze(0), out["wave2"].unsqueeze(0)]
    bits = torch.cat([torch.nn.functional.pad(p.contiguous().view(torch.int64), (0, pad)) for p in rows])
    bits = bits.reshape(8, -1, BLOCK)
    w = (2 * torch.arange(8 * BLOCK, dtype=torch.int64, device=bits.device) + 1).reshape(8, 1, BLOCK)
    return (bits * w).sum(dim=(0, 2))


def _worker(rank, world, port, n, ref_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), AKB_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from akbraytracing_amd import dist as AD
    from akbraytracing_amd.wavefront import RayWave, Shard
    AD.init_from_env()
    try:
        dev = torch.device("cuda", torch.cuda.current_device())
        shard = Shard.split(n, world, rank)
        rw = RayWave(_geom(), n, shard=shard, comm=AD.TorchComm(dev))
        out = rw.run()
        torch.cuda.synchronize()
        sums = block_checksums(out).cpu().numpy()
        b0 = shard.start // BLOCK
        ref_sums = np.load(os.path.join(ref_dir, "block_checksums.npy"))[b0:b0 + sums.shape[0]]
        ref_wave = np.load(os.path.join(ref_dir, "wave2.npy"), mmap_mode="r")
        lo, hi = shard.start, shard.start + shard.count
        wave = out["wave2"].cpu().numpy()
        res = {"rays": shard.count, "start": shard.start, "flags": list(out["flags"]), "blocks": int(sums.shape[0]),
               "blocks_equal": int(np.sum(sums == ref_sums)),
               "wave2_max_diff_nm": float(np.max(np.abs(wave - ref_wave[lo:hi]))),
               "wave2_nan": int(np.isnan(wave).sum())}
        # the faithful pupil and PSF of the sharded trace: no gather of the hits (faithful_dist.py)
        from test_faithful_dist_gpu import save_result
        from akbraytracing_amd.faithful_dist import ShardedFaithfulPupil
        sp = ShardedFaithfulPupil(n, AD.TorchComm(dev), slots=1)
        r, _ = sp.run(out["detcenter2"][1], out["detcenter2"][2], out["wave2"])
        if rank == 0:
            save_result(os.path.join(ref_dir, "faithful_8ranks.npz"), r)
        res["halo_rows"] = sp.plan.rows[1] - sp.plan.rows[0]
        res["band_vertices"] = sp.plan.band_count(rank)
        sp.close()
        with open(os.path.join(ref_dir, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_c4_1e8_rays_unsharded_and_eight_ranks(gpu, tmp_path):
    from akbraytracing_amd.wavefront import RayWave
    rw = RayWave(_geom(), N)
    out = rw.run()
    torch.cuda.synchronize()
    assert out["flags"] == (0, 0)
    assert out["opl"].shape[0] == N * N
    np.save(os.path.join(tmp_path, "block_checksums.npy"), block_checksums(out).cpu().numpy())
    wave = out["wave2"].cpu().numpy()
    assert not np.isnan(wave).any()
    np.save(os.path.join(tmp_path, "wave2.npy"), wave)
    # the faithful pupil and PSF of 1e8 hits on one GPU
    import time
    from akbraytracing_amd.faithful import FaithfulPupil
    from test_faithful_dist_gpu import KEYS, assert_same
    fp = FaithfulPupil(N, N, slots=2)
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        want = fp.run(out["detcenter2"][1], out["detcenter2"][2], out["wave2"])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
    print(f"C4 faithful pupil + PSF (1e8 hits -> 128^2 -> 2048^2), one process: {ms:.1f} ms")
    want = {k: want[k].clone() for k in KEYS}
    fp.close()
    assert np.isfinite(want["map"].cpu().numpy()).sum() > 0.5 * 128 * 128
    del rw, out, wave, fp
    torch.cuda.empty_cache()
    mp.start_processes(_worker, args=(WORLD, _free_port(), N, str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    res = [json.load(open(os.path.join(tmp_path, f"rank{r}.json"))) for r in range(WORLD)]
    assert sum(r["rays"] for r in res) == N * N
    assert all(abs(r["rays"] - N * N / WORLD) < 8192 for r in res)  # ~1250 V-rows per rank
    for r in res:
        assert r["flags"] == [0, 0]
        assert r["blocks_equal"] == r["blocks"], r  # pass 2 and Wave2 bit-exact, block by block
        assert r["wave2_nan"] == 0
        assert r["wave2_max_diff_nm"] == 0.0, r
    assert_same(os.path.join(tmp_path, "faithful_8ranks.npz"), want)
