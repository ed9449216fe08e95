"""numpy-exact sums on the device.

np.sum / np.mean / np.nanmean on a float64 row run numpy's pairwise summation inside 8192-element
buffers and add the buffer results left to right; akb_pairwise_sum_f64 reproduces that order, so
the means the drivers take (nanmean(arctan(...)) for the tilt, :3583-3588; mean(detcenter) :3590;
nanmean(totalDist) :3626/:3633; nanmean(detcenter) :3674) come out bit-identical to the reference.
"""
import torch

from . import _lib
from . import device as D


class RowSums:
    """Reusable workspace for row reductions of a (rows, n) float64 device tensor."""

    def __init__(self):
        self._work = None

    def __call__(self, x, nan=False, stream=None):
        """x: (rows, n) or (n,) contiguous float64 device tensor -> (sums, counts) device tensors."""
        L = _lib.lib()
        if x.dim() == 1:
            x = x.unsqueeze(0)
        if not x.is_contiguous():
            x = x.contiguous()
        rows, n = x.shape
        need = int(L.akb_pairwise_work_bytes(rows, n))
        if self._work is None or self._work.numel() * 8 < need or self._work.device != x.device:
            self._work = torch.empty(max(need // 8, 1), dtype=D.F64, device=x.device)
        sums = torch.empty(rows, dtype=D.F64, device=x.device)
        counts = torch.empty(rows, dtype=torch.int64, device=x.device)
        _lib.check(L.akb_pairwise_sum_f64(D.ptr(x), n, rows, n, int(bool(nan)), D.ptr(sums), D.ptr(counts),
                                          D.ptr(self._work), D.stream_handle(stream)))
        return sums, counts


_default = RowSums()


def np_sum(x, nan=False):
    """Device analogue of np.sum (nan=False) / np.nansum (nan=True) per row; returns (sums, counts)."""
    return _default(x, nan=nan)


def means_to_host(pairs):
    """[(sums, counts), ...] device tensors -> list of numpy float64 means, one sync.
    mean = sum / count in float64 (numpy's true_divide of the sum by the count)."""
    import numpy as np
    flat = [torch.cat([s, c.to(D.F64)]) for s, c in pairs]
    host = torch.cat(flat).cpu().numpy() if flat else np.zeros(0)
    out, off = [], 0
    for s, _ in pairs:
        r = s.shape[0]
        sums = host[off:off + r]
        cnts = host[off + r:off + 2 * r]
        with np.errstate(invalid="ignore", divide="ignore"):
            out.append(sums / cnts)
        off += 2 * r
    return out


class LeafSink:
    """Device buffers of an akb_leaf_sink: a producer kernel writes numpy pairwise leaf sums of
    nq per-element quantities, finish() completes them to np.sum / np.nanmean results."""

    def __init__(self, nq, n, nan_mask, dev):
        L = _lib.lib()
        self.nq, self.n = int(nq), int(n)
        nbytes = max(int(L.akb_leaf_sink_bytes(nq, n)), 256)
        self.buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.desc = _lib.LeafSink()
        _lib.check(L.akb_leaf_sink_layout(D.ptr(self.buf), nq, int(nan_mask), n, self.desc))
        wb = max(int(L.akb_leaf_finish_work_bytes(nq, n)), 16)
        self.work = torch.empty(wb // 8 + 1, dtype=D.F64, device=dev)
        self.sums = torch.empty(nq, dtype=D.F64, device=dev)
        self.counts = torch.empty(nq, dtype=torch.int64, device=dev)

    def finish(self, stream=None):
        L = _lib.lib()
        _lib.check(L.akb_leaf_finish_f64(self.desc, D.ptr(self.sums), D.ptr(self.counts), D.ptr(self.work),
                                         D.stream_handle(stream)))
        return self.sums, self.counts

    def finish_dist(self, comm, nbufs, n_total, stream=None):
        """finish() over ranks, bit for bit the single-process result: this rank's shard must be
        aligned to numpy's 8192-element buffers (wavefront.Shard.split), nbufs[r] the full buffers
        of rank r. Each rank forms its buffer sums and its short-buffer sum (only the last rank has
        one), one all-gather brings every rank's to every rank, and the buffer sums are added
        left to right in grid order, the short buffer last - numpy's order. The
        counts are integers: their all-reduced sum is exact. n_total: elements over all ranks.
        stream: a torch stream or a raw hipStream_t handle (default: the current stream); the
        kernels, the torch ops and the collective all run on it."""
        if stream is not None and not isinstance(stream, torch.cuda.Stream):
            h = D.stream_handle(stream).value or 0  # the null stream's handle is NULL
            if h != torch.cuda.current_stream().cuda_stream:
                stream = torch.cuda.ExternalStream(h)
            else:
                stream = None
        if stream is not None:
            with torch.cuda.stream(stream):
                return self.finish_dist(comm, nbufs, n_total)
        L = _lib.lib()
        nq, dev = self.nq, self.sums.device
        nb_max = max(max(nbufs), 1)
        sh = D.stream_handle()
        part = torch.zeros((nq, nb_max), dtype=D.F64, device=dev)
        pcnt = torch.zeros((nq, nb_max), dtype=torch.int64, device=dev)
        tsum = torch.empty(nq, dtype=D.F64, device=dev)
        tcnt = torch.empty(nq, dtype=torch.int64, device=dev)
        _lib.check(L.akb_leaf_parts_f64(self.desc, D.ptr(part), D.ptr(pcnt), nb_max, D.ptr(tsum), D.ptr(tcnt), sh))
        # one all-gather of everything (counts travel as float64: exact below 2^53)
        mine = torch.cat([part.reshape(-1), pcnt.reshape(-1).to(D.F64), tsum, tcnt.to(D.F64)])
        g = comm.allgather_equal(mine)  # (world, len)
        w = g.shape[0]
        m = nq * nb_max
        g_part = g[:, :m].reshape(w, nq, nb_max)
        g_pcnt = g[:, m:2 * m].reshape(w, nq, nb_max).to(torch.int64)
        tail = g[-1, 2 * m:2 * m + nq]  # the grid's short buffer lives on the last rank
        cnt_t = g[:, 2 * m + nq:].to(torch.int64).sum(dim=0)
        total = sum(nbufs)
        if total == 0:
            self.sums.copy_(tail)
            self.counts.copy_(cnt_t)
            return self.sums, self.counts
        parts = torch.cat([g_part[r, :, :nb] for r, nb in enumerate(nbufs) if nb], dim=1).contiguous()
        pcnts = torch.cat([g_pcnt[r, :, :nb] for r, nb in enumerate(nbufs) if nb], dim=1).contiguous()
        acc = torch.empty(nq, dtype=D.F64, device=dev)
        cnt = torch.empty(nq, dtype=torch.int64, device=dev)
        _lib.check(L.akb_parts_chain_f64(D.ptr(parts), D.ptr(pcnts), total, nq, total, D.ptr(acc), D.ptr(cnt), sh))
        # k_pw_final's acc + tail_sum: one IEEE add, the short buffer last
        self.sums.copy_(acc + tail if int(n_total) % 8192 != 0 else acc)
        self.counts.copy_(cnt + cnt_t)
        return self.sums, self.counts
