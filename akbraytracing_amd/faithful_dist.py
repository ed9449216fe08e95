"""The reference's pupil and PSF of a ray-sharded trace, without gathering the hits.

SURVEY.md §8(e) allowed gathering every rank's (y, z, Wave2) rows to one rank "until f1 replaces it
with a structured-grid method" (dist.wave_pupil_sharded: 24 B per ray, 2.4 GB at configs[3]'s 1e8
rays, and that one rank grids the whole lattice). The cone solve needs, for a target, only the
(2K + 4)^2 box of hits around its cell, or - near the lattice boundary, where the pocket chords
couple vertices along a whole side - the boundary band (akb_gd_cone_part_f64). So each rank keeps
its own rows:

  begin   its rows of (y, z, Wave2) into a window buffer, and the K + 3 rows on either side from
          the neighbouring ranks (point to point: 0.24 MB a row at 10000^2); the cell pass
          (diagonals, lattice checks) over the window; the boundary band - vertices of depth
          <= 2K + 3 and their cells: 1.2e6 of 1e8 hits at C4, 29 MB - to the band owner (rank
          `root`), which reads the ring and starts the pocket job (host, a worker thread);
  finish  the band owner's pockets to its device and the target axes from the ring, broadcast;
          every rank's claims over its own cell rows, MIN-reduced (the one-process claims are an
          atomicMin over all triangles); each rank forms the interior targets whose cell's first
          corner lies in its rays (LDS patches on its window), the band owner every band and
          pocket target (the band iteration); the pieces SUM-reduced to the band owner, which runs
          the one-workgroup post (nanmean, plane correction, psf_calc's rotation) and the PSF.

The map, pupil and PSF are the one-process FaithfulPupil's bit for bit (tests/test_c4_gpu.py: eight
ranks at 10000^2; tests/test_faithful_dist_gpu.py: 2 - 8 ranks at smaller grids). Collectives run
in the same order on every rank, so the caller decides when a run finishes, identically on all
ranks (a lag, not the band owner's pocket job). The plan and the data movement are plain torch and
run on CPU with gloo (tests/test_faithful_dist_cpu.py).
"""
import concurrent.futures
import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from .faithful import ErrorLog, cone_guard, pack_pockets
from .pupilmap import POST_PARAMS
from .griddata import CONE_SWEEPS, _F_NEG, _F_NONCONVEX, _F_NONFINITE, _F_NOT_DELAUNAY, _F_POCKET, _F_POS
from .wavefront import Shard

EUV = 13.5e-9


# ---------------------------------------------------------------------- the plan (host only)

def band_depth(K):
    """The band iteration's depth (akb_griddata.hip cone_part: 2K + 2); its vertices read one more."""
    return 2 * K + 2


def vertex_band_segments(lo, hi, n, depth):
    """[a, b) runs of the flat vertices iv * n + ih in [lo, hi) with min(iv, ih, n-1-iv, n-1-ih) <= depth."""
    out = []
    if hi <= lo:
        return out
    for r in range(lo // n, (hi - 1) // n + 1):
        a, b = r * n, (r + 1) * n
        if min(r, n - 1 - r) <= depth or 2 * (depth + 1) >= n:
            runs = [(a, b)]
        else:
            runs = [(a, a + depth + 1), (b - depth - 1, b)]
        for x, y in runs:
            x, y = max(x, lo), min(y, hi)
            if y > x:
                out.append((x, y))
    return out


def cell_band_segments(lo, hi, n, depth):
    """[a, b) runs of the cells iv * (n-1) + ih (iv, ih <= n-2) whose first corner iv * n + ih lies in
    [lo, hi) and min(iv, ih, n-2-iv, n-2-ih) <= depth."""
    out = []
    if hi <= lo:
        return out
    for r in range(lo // n, min((hi - 1) // n, n - 2) + 1):
        c_lo, c_hi = max(lo - r * n, 0), min(hi - r * n, n - 1)
        if c_hi <= c_lo:
            continue
        if min(r, n - 2 - r) <= depth or 2 * (depth + 1) >= n - 1:
            cols = [(0, n - 1)]
        else:
            cols = [(0, depth + 1), (n - 2 - depth, n - 1)]
        for x, y in cols:
            x, y = max(x, c_lo), min(y, c_hi)
            if y > x:
                out.append((r * (n - 1) + x, r * (n - 1) + y))
    return out


@dataclass
class ShardPlan:
    """Where rank `rank`'s data lives and what it exchanges, for K sweeps on an n x n lattice cut by
    Shard.split. Rows are lattice V-rows (iv); flat indices are global."""
    n: int
    world: int
    rank: int
    K: int
    root: int = 0
    shards: list = field(default_factory=list)
    own: tuple = (0, 0)    # my rays [start, end)
    claim: tuple = (0, 0)  # cell rows whose triangles I claim: every cell with its first corner in my rays
    rows: tuple = (0, 0)   # vertex rows my window holds: my rays' rows +- K + 3
    cells: tuple = (0, 0)  # cell rows of the cell pass: every cell a patch of mine reads
    base: int = 0          # first vertex row of my buffers (0 on the band owner: full-size buffers)
    nrows: int = 0
    halo_send: list = field(default_factory=list)  # (peer, a, b): my rays [a, b) that peer's window holds
    halo_recv: list = field(default_factory=list)  # (peer, a, b): peer's rays my window holds
    band_v: list = field(default_factory=list)     # per rank: its vertex band runs (depth <= 2K + 3)
    band_c: list = field(default_factory=list)     # per rank: its band cells' runs

    @staticmethod
    def make(n, world, rank, K=CONE_SWEEPS, root=0):
        n, world, rank, K = int(n), int(world), int(rank), int(K)
        p = ShardPlan(n, world, rank, K, root)
        p.shards = [Shard.split(n, world, r) for r in range(world)]
        wins = [ShardPlan._window(n, K, s) for s in p.shards]
        sh = p.shards[rank]
        p.own = (sh.start, sh.start + sh.count)
        p.claim, p.rows, p.cells = wins[rank]
        if rank == root:
            p.base, p.nrows = 0, n
        else:
            p.base, p.nrows = p.rows[0], p.rows[1] - p.rows[0]
        for i, (_, (R0, R1), _) in enumerate(wins):
            si = p.shards[i]
            need = [(R0 * n, si.start), (si.start + si.count, R1 * n)]
            for j, sj in enumerate(p.shards):
                if i == j:
                    continue
                for a, b in need:
                    a, b = max(a, sj.start), min(b, sj.start + sj.count)
                    if b > a:
                        if j == rank:
                            p.halo_send.append((i, a, b))
                        if i == rank:
                            p.halo_recv.append((j, a, b))
        d = band_depth(K) + 1
        p.band_v = [vertex_band_segments(s.start, s.start + s.count, n, d) for s in p.shards]
        p.band_c = [cell_band_segments(s.start, s.start + s.count, n, d) for s in p.shards]
        return p

    @staticmethod
    def _window(n, K, s):
        H = K + 3
        row0 = s.start // n
        row1 = min((s.start + s.count - 1) // n + 1, n - 1)
        R0, R1 = max(0, row0 - H), min(n, row1 + H + 1)
        # the cell pass reads the next row's cell too (its top edge): stop two rows short of R1
        c1 = n - 1 if R1 == n else R1 - 2
        return (row0, row1), (R0, R1), (R0, c1)

    @property
    def is_root(self):
        return self.rank == self.root

    def band_count(self, r):
        return sum(b - a for a, b in self.band_v[r])

    def cell_count(self, r):
        return sum(b - a for a, b in self.band_c[r])


def _index(runs, offset, dev):
    if not runs:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    return torch.cat([torch.arange(a - offset, b - offset, dtype=torch.int64, device=dev) for a, b in runs])


# ---------------------------------------------------------------------- data movement (torch only)

def _staged(comm, t):
    return comm._stage and t.is_cuda


def exchange_halo(plan, comm, vals, win, group=None):
    """vals: (C, count) my rays' rows; win: (C, nrows * n) my window. Copies my rays in and receives
    the halo rows from the neighbours (batched point to point; gloo + device tensors: staged)."""
    off = plan.base * plan.n
    a = plan.own[0] - off
    win[:, a:a + vals.shape[1]].copy_(vals)
    if plan.world == 1:
        return
    ops, back = [], []
    for peer, x, y in plan.halo_send:
        t = vals[:, x - plan.own[0]:y - plan.own[0]].contiguous()
        ops.append(dist.P2POp(dist.isend, t.cpu() if _staged(comm, t) else t, peer, group=group))
    for peer, x, y in plan.halo_recv:
        dst = win[:, x - off:y - off]
        buf = torch.empty(dst.shape, dtype=dst.dtype, device="cpu" if _staged(comm, win) else dst.device)
        ops.append(dist.P2POp(dist.irecv, buf, peer, group=group))
        back.append((buf, dst))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for buf, dst in back:
        dst.copy_(buf)


class BandGather:
    """Every rank's band (vertex values (C, .) and cell diagonals) into the band owner's full-size
    buffers: one gather of a padded piece per kind."""

    def __init__(self, plan, dev):
        self.plan = plan
        n = plan.n
        self.mv = max(plan.band_count(r) for r in range(plan.world))
        self.mc = max(max(plan.cell_count(r) for r in range(plan.world)), 1)
        self.my_v = _index(plan.band_v[plan.rank], plan.base * n, dev)
        self.my_c = _index(plan.band_c[plan.rank], plan.base * (n - 1), dev)
        if plan.is_root:
            self.all_v = [_index(plan.band_v[r], 0, dev) for r in range(plan.world)]
            self.all_c = [_index(plan.band_c[r], 0, dev) for r in range(plan.world)]

    def __call__(self, comm, win, diag, group=None):
        """win: (C, nrows * n) window values, diag: window diagonals (uint8). On the band owner
        (win, diag full size) the other ranks' band entries are written in place."""
        p = self.plan
        if p.world == 1:
            return
        C = win.shape[0]
        pv = torch.zeros((C, self.mv), dtype=win.dtype, device=win.device)
        pv[:, :self.my_v.shape[0]] = win[:, self.my_v]
        pc = torch.zeros(self.mc, dtype=torch.uint8, device=diag.device)
        pc[:self.my_c.shape[0]] = diag[self.my_c]
        if _staged(comm, win):
            pv, pc = pv.cpu(), pc.cpu()
        gv = [torch.empty_like(pv) for _ in range(p.world)] if p.is_root else None
        gc = [torch.empty_like(pc) for _ in range(p.world)] if p.is_root else None
        dist.gather(pv, gather_list=gv, dst=p.root, group=group)
        dist.gather(pc, gather_list=gc, dst=p.root, group=group)
        if not p.is_root:
            return
        for r in range(p.world):
            if r == p.rank:
                continue
            win[:, self.all_v[r]] = gv[r].to(win.device)[:, :self.all_v[r].shape[0]]
            diag[self.all_c[r]] = gc[r].to(diag.device)[:self.all_c[r].shape[0]]


def _collective(comm, t, fn):
    if comm.world == 1:
        return
    if _staged(comm, t):
        h = t.cpu()
        fn(h)
        t.copy_(h)
    else:
        fn(t)


def _broadcast(comm, t, root, group=None):
    _collective(comm, t, lambda x: dist.broadcast(x, src=root, group=group))


def _reduce_sum(comm, t, root, group=None):
    _collective(comm, t, lambda x: dist.reduce(x, dst=root, op=dist.ReduceOp.SUM, group=group))


def _all_reduce_min(comm, t, group=None):
    _collective(comm, t, lambda x: dist.all_reduce(x, op=dist.ReduceOp.MIN, group=group))


# ---------------------------------------------------------------------- the pipeline

class DistTicket:
    __slots__ = ("slot", "job", "npock", "err", "result", "h2d", "finished", "done", "erow")

    def ready(self):
        return self.job.done()


class ShardedFaithfulPupil:
    """The faithful pupil / PSF of runs traced as Shard.split row shards of an n x n grid: every rank
    calls begin / finish for the same runs in the same order (comm: dist.TorchComm). slots: runs
    between begin and finish."""

    def __init__(self, n, comm, size=128, pad=16, wavelengths=(EUV,), sweeps=CONE_SWEEPS, root=0, slots=2,
                 workers=2, delaunay_tol=1e-10):
        from . import _lib
        from . import device as D
        from .griddata import chebyshev_weights
        L = _lib.lib()
        self.comm = comm
        self.plan = p = ShardPlan.make(n, comm.world, comm.rank, sweeps, root)
        # a communicator of its own (every rank calls this constructor in the same order): the
        # trace's collectives on the other streams never queue behind these
        self.group = dist.new_group(list(range(comm.world))) if comm.world > 1 else None
        self.n, self.root, self.K = p.n, p.root, p.K
        self.dev = D.device()
        self.size, self.pad = int(size), int(pad)
        self.lams = [float(w) for w in wavelengths]
        self.tol = float(delaunay_tol)
        n = self.n
        m = self.size * self.size
        self.Lr = 4 * (n - 1)
        Lr, cap = self.Lr, self.Lr
        # the pocket block (FaithfulPupil's layout): tri | nbr | edge | xptr | xidx | npk
        self._o = dict(tri=0, nbr=3 * cap, edge=6 * cap, xptr=6 * cap + Lr, xidx=6 * cap + 2 * Lr + 1)
        self._o["npk"] = self._o["xidx"] + 6 * cap
        self.slots = []
        for _ in range(int(slots)):
            s = dict(win=torch.zeros((3, p.nrows * n), dtype=D.F64, device=self.dev),
                     diag=torch.zeros(max(p.nrows - 1, 1) * (n - 1), dtype=torch.uint8, device=self.dev),
                     flags=torch.zeros(1, dtype=torch.int32, device=self.dev),
                     rflags=torch.zeros(2 * comm.world, dtype=D.F64, device=self.dev), last=None)
            if p.is_root:
                s.update(ring=torch.zeros(2 * Lr + 1, dtype=D.F64, device=self.dev),
                         ring_host=torch.empty(2 * Lr + 1, dtype=D.F64, pin_memory=True),
                         pk_host=torch.zeros(self._o["npk"] + 1, dtype=torch.int32, pin_memory=True),
                         pk=torch.zeros(self._o["npk"] + 1, dtype=torch.int32, device=self.dev),
                         status=torch.zeros(1, dtype=torch.int64, device=self.dev))
            self.slots.append(s)
        self._next = 0
        self.band = BandGather(p, self.dev)
        self.work = torch.empty(int(L.akb_gd_cone_work_bytes(n, n, self.size, self.size, 1)) // 8 + 1, dtype=D.F64,
                                device=self.dev)
        self.owner = torch.empty(m, dtype=torch.int32, device=self.dev)
        self.axes = torch.zeros(2 * self.size + 6, dtype=D.F64, device=self.dev)  # gx | gy | extent | pitch
        # map piece | count | every rank's cell flags (slot r): one SUM reduction to the band owner
        # | every rank's cone error estimate (slot world + r)
        self.red = torch.zeros(2 * m + 2 * comm.world, dtype=D.F64, device=self.dev)
        self.map = torch.empty((1, self.size, self.size), dtype=D.F64, device=self.dev)
        self.change = torch.zeros(2, dtype=torch.int64, device=self.dev)  # change measure | value-error estimate
        self.post, self.psf = {}, None
        self._omegas = D.host_f64(chebyshev_weights(max(self.K, 1)))
        self.pool = concurrent.futures.ThreadPoolExecutor(max_workers=int(workers), thread_name_prefix="akb-pk") \
            if p.is_root else None
        self.flags_all = 0
        self._done = None  # the latest finish's end (finishes share work / owner / map / psf buffers)
        # per run (band owner): every rank's cell flags | the pocket status word | the post block's 18 words
        self.errors = ErrorLog(2 * comm.world + 1 + 2 + POST_PARAMS) if p.is_root else None
        self.finished = 0

    @staticmethod
    def _v(t, elems_off):
        """Device address of t minus elems_off elements: the windowed kernels index a virtual global
        array with global rows, and read only the rows this buffer backs."""
        return ctypes.c_void_p(t.data_ptr() - int(elems_off) * t.element_size())

    # ------------------------------------------------------------------ stage 1
    def begin(self, y, z, f, stream=None):
        """y, z, f: this rank's rows (its Shard's rays) of detcenter2[1], [2] and Wave2 (device).
        Returns a DistTicket."""
        from . import _lib
        from . import device as D
        L = _lib.lib()
        p, n = self.plan, self.n
        if y.shape[0] != p.own[1] - p.own[0]:
            raise ValueError(f"rank {p.rank} holds rays [{p.own[0]}, {p.own[1]}): got {y.shape[0]} rows")
        s = self.slots[self._next]
        self._next = (self._next + 1) % len(self.slots)
        if s["last"] is not None:
            prev = s["last"]
            if not prev.finished:
                raise RuntimeError("ShardedFaithfulPupil: more runs begun than slots before a finish")
            if prev.h2d is not None:
                prev.h2d.synchronize()
        st = torch.cuda.current_stream() if stream is None else stream
        sh = D.stream_handle(st)
        win, diag = s["win"], s["diag"]
        t = DistTicket()
        t.slot, t.npock, t.err, t.result, t.h2d, t.finished, t.done, t.erow = s, 0, None, None, None, False, None, None
        with torch.cuda.stream(st):
            if s["last"] is not None and s["last"].done is not None:  # the slot's last reader
                st.wait_event(s["last"].done)
            for a in (y, z, f):  # read on this stream (the trace allocated them on its own)
                a.record_stream(st)
            exchange_halo(p, self.comm, torch.stack([y, z, f]), win, self.group)
            off = p.base * n
            s["flags"].zero_()
            _lib.check(L.akb_gd_cells_window_f64(self._v(win[0], off), self._v(win[1], off), n, n, p.cells[0],
                                                 p.cells[1], self._v(diag, p.base * (n - 1)), self.tol,
                                                 D.ptr(s["flags"]), sh))
            self.band(self.comm, win, diag, self.group)
            if p.is_root:
                Lr = self.Lr
                ring = s["ring"]
                ring[2 * Lr:].zero_()
                rflags = ring.view(torch.int32)[4 * Lr:4 * Lr + 1]
                _lib.check(L.akb_gd_ring_f64(D.ptr(win[0]), D.ptr(win[1]), n, n, D.ptr(ring[:Lr]),
                                             D.ptr(ring[Lr:2 * Lr]), D.ptr(rflags), sh))
                s["ring_host"].copy_(ring, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                t.job = self.pool.submit(self._pockets, s, ev)
            else:
                t.job = concurrent.futures.Future()
                t.job.set_result((0, None))
        s["last"] = t
        return t

    def _pockets(self, s, ev):
        """Worker thread on the band owner: the pockets from the ring. An error comes back as a value
        (every rank still runs finish's collectives) with the pocket block left empty."""
        from . import _lib
        ev.synchronize()
        L = _lib.lib()
        Lr, o = self.Lr, self._o
        buf = s["pk_host"].numpy()
        try:
            rb = s["ring_host"].numpy()
            if int(rb[2 * Lr:].view(np.int32)[0]) & _F_NONFINITE:
                raise ValueError("griddata: non-finite point coordinates (a ray that missed)")
            hp = lambda k: buf[o[k]:].ctypes.data_as(_lib.c_vp)  # noqa: E731
            _lib.check(L.akb_gd_pockets(rb[:Lr].ctypes.data_as(_lib.c_vp), rb[Lr:2 * Lr].ctypes.data_as(_lib.c_vp),
                                        self.n, self.n, Lr, hp("npk"), hp("tri"), hp("nbr"), hp("edge"), hp("xptr"),
                                        hp("xidx")))
            npk, s["po"] = pack_pockets(buf, o, Lr)
            return npk, None
        except Exception as e:  # noqa: BLE001 - raised again by check()
            buf[o["edge"]:o["edge"] + Lr] = -1  # no pocket neighbours and no chords: every index in range
            buf[o["xptr"]:o["xptr"] + Lr + 1] = 0
            buf[o["npk"]] = 0
            _, s["po"] = pack_pockets(buf, o, Lr)
            return 0, e

    # ------------------------------------------------------------------ stage 2
    def finish(self, t, stream=None, events=None, psf_events=None):
        """Queue the rest of t's chain. Returns dict(psf, map, corrected, rotated, params, axes,
        change) on the band owner, None elsewhere. events / psf_events: optional (start, end)
        timing events around the device work / the PSF alone (band owner)."""
        from . import _lib
        from . import device as D
        from .psf import psf_stack
        from .pupilmap import pupil_post
        L = _lib.lib()
        p, n, m, K = self.plan, self.n, self.size, self.K
        t.npock, t.err = t.job.result()
        s = t.slot
        st = torch.cuda.current_stream() if stream is None else stream
        sh = D.stream_handle(st)
        win, diag = s["win"], s["diag"]
        off = p.base * n
        vx, vy, vf = self._v(win[0], off), self._v(win[1], off), self._v(win[2], off)
        vd = self._v(diag, p.base * (n - 1))
        gx, gy = self.axes[:m], self.axes[m:2 * m]
        mm = m * m
        red = self.red
        with torch.cuda.stream(st):
            if self._done is not None:  # the shared buffers' last finish, on any stream
                st.wait_event(self._done)
            if events is not None:
                events[0].record(st)
            if p.is_root:
                o, Lr = s["po"], self.Lr
                pk = s["pk"]
                pk[:o["len"]].copy_(s["pk_host"][:o["len"]], non_blocking=True)
                t.h2d = torch.cuda.Event()
                t.h2d.record(st)
                pock = (t.npock, D.ptr(pk[o["tri"]:]), D.ptr(pk[o["nbr"]:]), D.ptr(pk[o["edge"]:]))
                chords = (D.ptr(pk[o["xptr"]:]), D.ptr(pk[o["xidx"]:]))
                s["status"].zero_()
                _lib.check(L.akb_gd_check_pockets(vx, vy, n, n, vd, *pock, self.tol, D.ptr(s["status"]), sh))
                ring = s["ring"]
                _lib.check(L.akb_gd_axes_f64(D.ptr(ring[:Lr]), D.ptr(ring[Lr:2 * Lr]), Lr, m, m, D.ptr(gx),
                                             D.ptr(gy), D.ptr(self.axes[2 * m:]), sh))
            else:
                pock, chords = (0, None, None, None), (None, None)
            _broadcast(self.comm, self.axes, p.root, self.group)
            _lib.check(L.akb_gd_claims_f64(vx, vy, n, n, vd, *pock, p.claim[0], p.claim[1], int(p.is_root),
                                           D.ptr(gx), m, D.ptr(gy), m, D.ptr(self.owner), D.ptr(self.work), sh))
            _all_reduce_min(self.comm, self.owner, self.group)
            self.change.zero_()
            _lib.check(L.akb_gd_cone_part_f64(vx, vy, n, n, vd, *pock, *chords, p.own[0], p.own[1], int(p.is_root),
                                              D.ptr(gx), m, D.ptr(gy), m, vf, 1, K, self._omegas, D.ptr(self.work),
                                              D.ptr(self.owner), D.ptr(red[:mm]), D.ptr(red[mm:2 * mm]),
                                              D.ptr(self.change), sh))
            red[2 * mm:].zero_()
            red[2 * mm + p.rank] = s["flags"][0].to(D.F64)
            red[2 * mm + self.comm.world + p.rank] = self.change.view(D.F64)[1]
            _reduce_sum(self.comm, red, p.root, self.group)
            res = None
            if p.is_root:
                s["rflags"].copy_(red[2 * mm:])
                self.map.view(-1).copy_(red[:mm])
                _lib.check(L.akb_gd_part_finish_f64(D.ptr(self.map), D.ptr(red[mm:2 * mm]), mm, 1, sh))
                post = pupil_post(self.map[0], out=self.post, stream=st)
                self.post = post
                if psf_events is not None:
                    psf_events[0].record(st)
                psf, _, _ = psf_stack(post["opd"], None, self.lams, None, pad_factor=self.pad, stream=st,
                                      out=self.psf, pitch=self.axes[2 * m + 4:2 * m + 6])
                if psf_events is not None:
                    psf_events[1].record(st)
                self.psf = psf
                res = dict(psf=psf, map=self.map[0], corrected=post["corrected"], rotated=post["rotated"],
                           params=post["params"], axes=self.axes, change=self.change)
                t.erow = self.errors.record((s["rflags"], s["status"].view(D.F64), self.change.view(D.F64),
                                             post["params"]), st)  # rflags: the flags | the estimates
            if events is not None:
                events[1].record(st)
            t.done = torch.cuda.Event()
            t.done.record(st)
            self._done = t.done
        t.result = res
        t.finished = True
        self.finished += 1
        return res

    def check(self, t):
        """Raise as the one-process chain would (band owner; waits for the device): non-finite hits, a
        lattice that is not a convex unfolded grid, pockets that are not locally Delaunay, too few
        points for the plane fits. The other ranks hold no result and return. Reads t's own error
        words (faithful.ErrorLog), not the slot's current ones."""
        from . import _lib
        from .pupilmap import pupil_post_check
        if not self.plan.is_root:
            return
        if t.err is not None:
            raise t.err
        if t.erow is None:
            return
        w = self.errors.read(*t.erow, t.done)
        world = self.comm.world
        fl = 0
        for v in w[:world]:
            fl |= int(v)
        est = float(np.max(w[world:2 * world]))  # every rank's interior targets
        w = np.concatenate([w[:world], w[2 * world:]])
        self.flags_all = fl
        if fl & _F_NONFINITE:
            raise ValueError("griddata: non-finite point coordinates (a ray that missed)")
        if fl & _F_NONCONVEX or (fl & _F_POS and fl & _F_NEG):
            raise _lib.AKBError("griddata: the points do not form a convex, unfolded lattice")
        if fl & _F_NOT_DELAUNAY:
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
        if int(w[world:world + 1].view(np.int64)[0]) & (_F_NOT_DELAUNAY | _F_POCKET):
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
        pupil_post_check(w[world + 3:])
        cone_guard(est, w[world + 3:])

    def run(self, y, z, f, stream=None):
        """begin + finish + check of one run: (result or None, ticket). The band owner's guard verdict
        is broadcast, so every rank takes the same path: a run whose cone solve fails its guard
        (ConeNotConverged; FaithfulPupil.run's fallback) is formed again from the converged gradients -
        the ranks' hits gathered to the band owner, which grids the whole lattice with the global
        sweeps to scipy's tolerance on the run's axes; the other ranks return None, as for every
        run. Any other error raises on the band owner only (after the run's collectives, so the
        group stays in step)."""
        from .griddata import ConeNotConverged
        t = self.begin(y, z, f, stream)
        res = self.finish(t, stream)
        verdict, err = 0, None
        if self.plan.is_root:
            try:
                self.check(t)
            except ConeNotConverged as e:
                verdict, err = 1, e
            except BaseException as e:  # raised below, after the verdict's collective
                verdict, err = 2, e
        v = torch.tensor([float(verdict)], dtype=torch.float64, device=self.dev)
        _broadcast(self.comm, v, self.plan.root, self.group)
        verdict = int(v.item())
        if verdict == 1:
            res = self._converged(y, z, f, stream)
        elif verdict == 2 and err is not None:
            raise err
        return res, t

    def _converged(self, y, z, f, stream=None):
        """The guard's fallback (collective): every rank's rows to the band owner, which forms the
        run's map from the global gradient iteration (CubicGrid.interp) on the run's axes, then the
        same post and PSF; None on the other ranks."""
        from . import device as D
        from .dist import gather_to_root
        from .griddata import CubicGrid
        from .pupilmap import pupil_post, pupil_post_check
        from .psf import psf_stack
        p, m = self.plan, self.size
        counts = [sh.count for sh in p.shards]
        got = gather_to_root(self.comm, [y.contiguous(), z.contiguous(), f.contiguous()], counts, p.root)
        if got is None:
            return None
        st = torch.cuda.current_stream() if stream is None else stream
        with torch.cuda.stream(st):
            ya, za, fa = got
            cg = CubicGrid(ya, za, self.n, self.n, delaunay_tol=self.tol)
            self.map[0].copy_(cg.interp(fa.reshape(1, -1), self.axes[:m], self.axes[m:2 * m])[0])
            post = pupil_post(self.map[0], out=self.post, stream=st)
            self.post = post
            psf, _, _ = psf_stack(post["opd"], None, self.lams, None, pad_factor=self.pad, stream=st,
                                  out=self.psf, pitch=self.axes[2 * m + 4:2 * m + 6])
            self.psf = psf
            self._done = torch.cuda.Event()  # the shared buffers' last writer (see FaithfulPupil._converged)
            self._done.record(st)
        pupil_post_check(post["params"])
        return dict(psf=psf, map=self.map[0], corrected=post["corrected"], rotated=post["rotated"],
                    params=post["params"], axes=self.axes, change=self.change, converged=True)

    def close(self):
        if self.pool is not None:
            self.pool.shutdown(wait=True)
