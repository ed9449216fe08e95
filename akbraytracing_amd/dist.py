"""One process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm; "gloo" on CPU).

The hot path shards without a data-path collective:
  * ray trace: each rank owns a contiguous block of V-rows of the ray grid (Shard.split); the
    only exchanges are the 2n resample samples (middle row / middle column picks), the flag
    word, a handful of partial sums for the means, and the assembled pupil before the PSF
    (SURVEY.md §5, §8(e));
  * Huygens: targets are split across ranks, sources replicated, and the new field is
    all-gathered so it can serve as the next stage's source set (Wavecalc _multi.py:136-138,
    :228, as a collective instead of peer reads).

The reference has no collectives at all (its multi-GPU code is CuPy device contexts + threads).
"""
import os

import numpy as np
import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default group from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            # AKB_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin,
            # collectives staged through the host); the default is RCCL, one rank per GPU
            backend = os.environ.get("AKB_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        elif torch.cuda.is_available():
            torch.cuda.set_device(local % torch.cuda.device_count())
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


class TorchComm:
    """Communicator for RayWave over the default process group."""

    def __init__(self, device=None):
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.device = device
        # gloo with device tensors (a rehearsal of the RCCL path): stage through host memory
        self._stage = dist.is_initialized() and dist.get_backend() == "gloo"

    def _dev(self, t):
        return t if self.device is None else t.to(self.device)

    def _all_reduce(self, t, op):
        t = t.contiguous()
        if self._stage and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)
        return t

    def allreduce_sums(self, t):
        if self.world > 1:
            t = self._all_reduce(t, dist.ReduceOp.SUM)
        return t

    def allreduce_max(self, t):
        if self.world > 1:
            t = self._all_reduce(t, dist.ReduceOp.MAX)
        return t

    def allgather_equal(self, t):
        """(world, *t.shape): every rank's t (same shape on every rank), in rank order."""
        if self.world == 1:
            return t.unsqueeze(0)
        t = t.contiguous()
        if self._stage and t.is_cuda:
            return self.allgather_equal(t.cpu()).to(t.device)
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t) if hasattr(dist, "all_gather_into_tensor") and t.is_cuda else \
            dist.all_gather(list(out.unbind(0)), t)
        return out

    def gather_samples(self, samp_h, samp_v, shard, n):
        """Each rank holds zeros outside its rows; one SUM all-reduce assembles both pick lists."""
        if self.world == 1:
            return samp_h, samp_v
        buf = self._dev(torch.from_numpy(np.concatenate([samp_h, samp_v])))
        buf = self.allreduce_sums(buf).cpu().numpy()
        return buf[:samp_h.shape[0]], buf[samp_h.shape[0]:]

    def allreduce_or(self, words):
        """Bitwise OR of int32 flag words over ranks, in place. RCCL has no bitwise reduction, so
        each word is unpacked to its 32 bits, the bits are MAX-reduced and packed again (a SUM
        would carry: two ranks' FLAG_MISS 0x1 would read as FLAG_ZERO_NORMAL 0x2)."""
        if self.world == 1:
            return words
        shifts = torch.arange(32, dtype=torch.int64, device=words.device)
        bits = (words.to(torch.int64).unsqueeze(-1) >> shifts) & 1
        bits = self._all_reduce(bits.contiguous(), dist.ReduceOp.MAX)
        packed = (bits << shifts).sum(-1)
        words.copy_(torch.where(packed >= 2 ** 31, packed - 2 ** 32, packed).to(words.dtype))
        return words

    def or_flags(self, f):
        """One host flag word OR-ed over ranks."""
        if self.world == 1:
            return f
        t = self._dev(torch.tensor([int(f)], dtype=torch.int32))
        return int(self.allreduce_or(t).item())

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def gather_field(self, piece, counts, root=0):
        """Concatenate per-rank 1-D pieces (lengths `counts`) in rank order on `root` (None on the
        other ranks): one gather, each rank's piece crossing the links once."""
        if self.world == 1:
            return piece
        if self._stage and piece.is_cuda:
            got = self.gather_field(piece.cpu(), counts, root)
            return got.to(piece.device) if got is not None else None
        mx = max(counts)
        pad = torch.zeros(mx, dtype=piece.dtype, device=piece.device)
        pad[:piece.shape[0]] = piece
        real = (lambda t: torch.view_as_real(t)) if pad.is_complex() else (lambda t: t)
        bufs = [torch.empty_like(pad) for _ in range(self.world)] if self.rank == root else None
        dist.gather(real(pad), gather_list=[real(b) for b in bufs] if bufs is not None else None, dst=root)
        if self.rank != root:
            return None
        return torch.cat([b[:c] for b, c in zip(bufs, counts)])

    def allgather_field(self, piece, counts):
        """Concatenate per-rank 1-D pieces (lengths `counts`) in rank order on every rank."""
        if self.world == 1:
            return piece
        mx = max(counts)
        pad = torch.zeros(mx, dtype=piece.dtype, device=piece.device)
        pad[:piece.shape[0]] = piece
        if self._stage and pad.is_cuda:
            return self.allgather_field(piece.cpu(), counts).to(piece.device)
        bufs = [torch.empty_like(pad) for _ in range(self.world)]
        if pad.is_complex():
            real = [torch.view_as_real(b) for b in bufs]
            dist.all_gather(real, torch.view_as_real(pad))
        else:
            dist.all_gather(bufs, pad)
        return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def gather_to_root(comm, pieces, counts, root=0):
    """Concatenate each rank's 1-D pieces (a list of same-length tensors per rank; rank r holds
    counts[r] elements) in rank order on `root` only: a list of full tensors there, None elsewhere.
    SURVEY.md §8(e)'s route for the global griddata step: the (y, z, Wave2) triples of every shard
    meet on one rank (24 B per ray: 2.4 GB at configs[3]'s 1e8 rays). gloo: staged through host
    memory."""
    if comm.world == 1:
        return list(pieces)
    out = [comm.gather_field(p, counts, root) for p in pieces]
    return out if comm.rank == root else None


def wave_pupil_sharded(rw, out, size, comm, root=0):
    """The faithful pupil (pupilmap.wave_pupil) of a ray-sharded trace: each rank hands its rows of
    detcenter2 (y, z) and Wave2 to `root` (gather_to_root), which grids the whole n x n lattice.
    Returns wave_pupil's tuple on root, None elsewhere."""
    from .pupilmap import wave_pupil
    counts = [int(c) for c in comm.allgather_equal(
        torch.tensor([rw.shard.count], dtype=torch.int64, device=out["wave2"].device)).reshape(-1).tolist()]
    d2 = out["detcenter2"]
    got = gather_to_root(comm, [d2[1].contiguous(), d2[2].contiguous(), out["wave2"].contiguous()], counts, root)
    if got is None:
        return None
    y, z, w = got
    return wave_pupil((y, z), w, rw.n, rw.n, grid_num_H=size, grid_num_V=size)


def split_counts(n, world):
    base, rem = divmod(n, world)
    return [base + (1 if r < rem else 0) for r in range(world)]


def propagate_sharded(tx, ty, tz, sx, sy, sz, u_ds, k, comm, propagate=None, splits=None):
    """Huygens stage with targets split over ranks (np.array_split order) and the result
    all-gathered. tx.. are the FULL target arrays (device tensors) on every rank. Every rank sums
    its sources in the whole problem's split order (splits: that count, default the library's for
    the full sizes), so the gathered field is the one-process field bit for bit. propagate: the
    per-rank kernel call (default wavecalc.propagate)."""
    from . import wavecalc as W
    n = int(tx.shape[0])
    if propagate is None:
        propagate = W.propagate
        if splits is None:
            splits = W.splits_for(n, int(sx.shape[0]))
    counts = split_counts(n, comm.world)
    lo = sum(counts[:comm.rank])
    hi = lo + counts[comm.rank]
    kw = {} if splits is None else {"splits": splits}
    piece = propagate(tx[lo:hi].contiguous(), ty[lo:hi].contiguous(), tz[lo:hi].contiguous(), sx, sy, sz, u_ds, k,
                      **kw)
    return comm.allgather_field(piece, counts)


def wavelength_shard(wavelengths, world, rank):
    """SURVEY.md §8(e) PSF stack sharding: rank r transforms wavelengths[r::world] - one wavelength
    per GPU for config 5's three at N >= 3, everything on rank 0 at N = 1, nothing on ranks beyond
    the stack. Every rank holds the whole pupil (RayWave.pupil all-reduces it)."""
    return list(wavelengths)[rank::world]


def psf_stack_sharded(opd, wavelengths, comm, gather=False, **kw):
    """psf_stack over this rank's wavelength_shard. Returns (psf (B_r, py, px) or None, the
    wavelengths it holds); gather=True all-gathers the whole (B, py, px) stack in wavelength order
    on every rank instead (B * py * px * 8 bytes over the links: an on-demand step, not per trace)."""
    from .psf import psf_stack
    lams = list(wavelengths)
    mine = wavelength_shard(lams, comm.world, comm.rank)
    psf = psf_stack(opd, None, mine, None, **kw)[0] if mine else None
    if not gather or comm.world == 1:
        return psf, mine
    ny, nx = int(opd.shape[0]), int(opd.shape[1])
    pad = int(kw.get("pad_factor", 2))
    plane = ((ny + ny % 2) * pad) * ((nx + nx % 2) * pad)
    counts = [len(wavelength_shard(lams, comm.world, r)) * plane for r in range(comm.world)]
    piece = psf.reshape(-1) if psf is not None else torch.zeros(0, dtype=torch.float64, device=opd.device)
    flat = comm.allgather_field(piece, counts)
    py, px = (ny + ny % 2) * pad, (nx + nx % 2) * pad
    out = torch.empty((len(lams), py, px), dtype=torch.float64, device=opd.device)
    off = 0
    for r in range(comm.world):
        for j, _ in enumerate(wavelength_shard(lams, comm.world, r)):
            out[r + j * comm.world] = flat[off:off + plane].reshape(py, px)
            off += plane
    return out, lams
