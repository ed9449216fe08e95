"""The wavefront hot path of the AKB / KB drivers, device-resident.

One call of RayWave.run() is what plot_result_debug(params, 'ray_wave') does between setting up
its mirrors and calling griddata (AKB_raytrace_20250312.py:2675-3689), on an n x n ray grid:

  pass 1    fused chain over the grid, exit slopes of the middle row/column     :2770-2845
  resample  np.arctan + interp1d (restated in C) + np.tan on the host (2n values) :2849-2879
  pass 2    fused chain + OPL + pre-tilt detector + arctan of the exit slopes   :2881-2905
  means     numpy-exact device sums -> theta_y, theta_z, focus_apprx, R_y, R_z  :3583-3591, :917-927
  tilt      rotate direction / last hit (dgemm FMA order), detectors 1 and 2,
            totalDist, totalDist2                                               :3592-3633
  OPD       DistError2, Sph, Wave2 = DistError2 - Sph                           :3626-3677

The same object serves KB_debug (2 mirrors, :10948-11054) and any quadric chain. Geometry is
a SystemGeometry: the mirrors in trace order, detector planes and the ray-grid angle ranges.
Multi-GPU: pass a Shard (contiguous V-rows of the grid) and a communicator (see dist.py); the
only exchanges are the 2n resample samples, a handful of means and the flag word.
"""
import json
import dataclasses
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import device as D
from . import primitives as P
from .reduce import LeafSink, RowSums
from .trace import ChainLaunch, Mirror, _fill_desc, staged_chain


@dataclass
class AngleRange:
    start: float
    stop: float
    offset: float

    def table(self, n):
        """rand_p0 = linspace(start, stop, n) - offset (AKB_raytrace_20250312.py:2695-2698)."""
        return np.linspace(self.start, self.stop, n) - np.float64(self.offset)


@dataclass
class SystemGeometry:
    mirrors: list
    det1: list                      # detector plane (g, h, i, j) at s2f_middle + defocus
    angle_h: AngleRange
    angle_v: AngleRange
    det2: list = None               # detector plane at + defocusWave ('ray_wave')
    source: tuple = (0.0, 0.0, 0.0)
    name: str = ""
    meta: dict = field(default_factory=dict)

    @staticmethod
    def from_dict(d):
        def plane(p):
            if p is None:
                return None
            p = [float(x) for x in p]
            return p[6:10] if len(p) == 10 else p
        return SystemGeometry(
            mirrors=[Mirror(m["coeffs"], m.get("negative", False)) for m in d["mirrors"]],
            det1=plane(d["det1"]), det2=plane(d.get("det2")),
            angle_h=AngleRange(**d["angle_h"]), angle_v=AngleRange(**d["angle_v"]),
            source=tuple(d.get("source", (0.0, 0.0, 0.0))), name=d.get("name", ""), meta=d.get("meta", {}))

    @staticmethod
    def load(path):
        with open(path) as f:
            return SystemGeometry.from_dict(json.load(f))


NP_BUF = 8192  # numpy's float64 sum buffer: pairwise inside, buffers added left to right


@dataclass
class Shard:
    """Contiguous block [start, start + count) of the n x n ray grid's flat rays (iv * n + ih, V-row
    major). Shard.split cuts the grid at multiples of numpy's 8192-element sum buffers, so every
    shard but the last holds whole buffers and the grid's short last buffer lies in the last one:
    each rank's buffer sums are then numpy's own and the means combine across ranks in numpy's
    order, bit for bit (reduce.LeafSink.finish_dist)."""
    start: int
    count: int

    @staticmethod
    def split(n, world, rank):
        """Rank `rank`'s contiguous range of whole 8192-ray numpy sum buffers (the last rank takes the
        short tail buffer too), so N ranks' per-buffer sums chain into one process's bits. A grid
        needs at least 8192 * world rays to split (the reference's 33^2 / 65^2 grids run on one
        rank): below that this raises ValueError, before any RayWave is built."""
        total = int(n) * int(n)
        if world == 1:
            return Shard(0, total)
        nbuf = total // NP_BUF
        if nbuf < world:
            raise ValueError(f"a {n} x {n} grid holds {nbuf} full 8192-ray buffers: too few for {world} ranks "
                             f"(row shards need at least {NP_BUF * world} rays; trace it on one rank)")
        base, rem = divmod(nbuf, world)
        b0 = rank * base + min(rank, rem)
        nb = base + (1 if rank < rem else 0)
        start = b0 * NP_BUF
        end = total if rank == world - 1 else (b0 + nb) * NP_BUF
        return Shard(start, end - start)

    def full_buffers(self):
        return self.count // NP_BUF


def geometry_key(g):
    """What a chain launch takes from a SystemGeometry (mirrors, pre-tilt detector, source):
    equal keys trace identically."""
    return (tuple(tuple(m.coeffs) + (bool(m.negative),) for m in g.mirrors), tuple(float(x) for x in g.det1),
            tuple(float(x) for x in g.source))


def sample_plan(n):
    """Indices of the equal-angle resample picks (:2851-2856): column round((n-1)/2) and the flat
    range [round(n(n-1)/2), round(n(n+1)/2))."""
    col = round((n - 1) / 2)
    return round(n * (n - 1) / 2), round(n * (n + 1) / 2), col


def sample_ownership(shard, n):
    """Which resample picks a shard's rays supply: (mask over the middle-row range, mask over the
    n rows of the middle column)."""
    hb, he, col = sample_plan(n)
    lo, hi = shard.start, shard.start + shard.count
    own_h = np.zeros(he - hb, dtype=bool)
    own_h[max(lo, hb) - hb:max(min(hi, he) - hb, 0)] = True
    g = np.arange(n) * n + col
    own_v = (g >= lo) & (g < hi)
    return own_h, own_v


def resample_axis(angle_sep, rand, out=None):
    """interp1d(angle_sep, rand, kind='linear')(np.linspace(angle_sep[0], angle_sep[-1], n)) — one
    axis of :2861-2870, done by the library's host routine (numpy linspace / interp and scipy's
    stable sort restated; ValueError out of range like interp1d)."""
    x = np.ascontiguousarray(angle_sep, dtype=np.float64)
    y = np.ascontiguousarray(rand, dtype=np.float64)
    if x.ndim != 1 or x.shape != y.shape:
        raise ValueError("resample needs two 1-D arrays of one length")
    if out is None:
        out = np.empty_like(x)
    L = _lib.lib()
    if L.akb_resample_f64(x.ctypes.data, y.ctypes.data, x.shape[0], out.ctypes.data) != 0:
        raise ValueError(L.akb_last_error().decode())
    return out


def resample(angle_h_sep, angle_v_sep, rand_h, rand_v):
    """:2861-2870 — interp1d of the launch angles onto equally spaced exit angles."""
    return resample_axis(angle_h_sep, rand_h), resample_axis(angle_v_sep, rand_v)


class RunResult(dict):
    """RayWave.run()'s outputs. theta_y, theta_z and focus_apprx live in the device parameter
    block of the tilt; they are copied to the host on first access (the run itself never waits
    for them)."""
    _LAZY = ("theta_y", "theta_z", "focus_apprx")

    def __init__(self, *a, params=None, **k):
        super().__init__(*a, **k)
        self._params = params
        self._host = None

    def tilt_params(self):
        """Host copy of the tilt's device parameter block: theta_y, theta_z, R_y (3 x 3, row-major),
        R_z, the focus estimate, the flag words (akb_tilt_params_f64); None for a run that took
        the staged path (host-formed matrices)."""
        if self._host is None and self._params is not None:
            self._host = self._params.cpu().numpy()
        return self._host

    def _resolve(self):
        h = self.tilt_params()
        if h is not None and "theta_y" not in dict.keys(self):
            self._params = None
            dict.update(self, theta_y=np.float64(h[0]), theta_z=np.float64(h[1]), focus_apprx=h[20:23].copy())

    def __getitem__(self, k):
        if k in self._LAZY:
            self._resolve()
        return dict.__getitem__(self, k)

    def get(self, k, default=None):
        return self[k] if k in self else default

    def __contains__(self, k):
        return (k in self._LAZY and self._params is not None) or dict.__contains__(self, k)


class LocalComm:
    """Single-process communicator (world of one)."""
    world = 1
    rank = 0

    def gather_samples(self, samp_h, samp_v, shard, n):
        return samp_h, samp_v

    def or_flags(self, f):
        return f

    def allreduce_or(self, words):
        return words

    def allgather_equal(self, t):
        return t.unsqueeze(0)

    def allreduce_sums(self, t):
        return t

    def allreduce_max(self, t):
        return t


@dataclass
class _Front:
    """What launch_front hands to launch_back."""
    r: object
    tan_h2: torch.Tensor
    tan_v2: torch.Tensor
    params: torch.Tensor
    full: bool
    stream: object
    flags: tuple = None  # (pass 1, pass 2) trace flag words once known (RayWave._resolve)
    flag_ev: object = None  # event after the flag words' copy to the host
    done: object = None  # event on the front's stream after its last kernel (the tilt parameters)
    slot: int = 0  # which of the per-run buffer sets (tables, extent keys, tilt sink) this run uses
    tilt: dict = None  # tilt outputs, when the next front's pass 1 already tilted this run (fused)
    tilted: object = None  # event after that fused kernel
    fin: tuple = None  # (sums, counts) of the fused tilt's sink, finished on RayWave._fin
    fin_ev: object = None  # event after that finish
    opd: dict = None  # DistError2 / Wave2, when the front after next formed them in its pass 1
    opd_ev: object = None  # event after that fused kernel
    g: object = None  # the SystemGeometry this run traced (RayWave.launch_front(geometry=...))


class RayWave:
    """Device-resident 'ray_wave' / 'wave' trace on an n x n grid (one shard of it).

    Every launch is prepared once (descriptors, device buffers, pinned host staging). A run
    waits on the host once, for the resample picks of pass 1 (the resample itself is host work
    by design, see resample_axis); pass 2, the tilt parameters, the tilt and the OPD are queued
    back to back, and the run returns as soon as pass 2's flag word has reached the host."""

    NSLOTS = 4  # runs in flight: k (front), k-1 (its sums finishing), k-2 (tilt fused into k), k-3 (OPD fused into k)

    def __init__(self, geometry, n, shard=None, comm=None, resample_pass=True, perturbation=None):
        """perturbation: optional legendre.LegendrePerturbation added to every ray's pass-2 optical
        path (BASELINE config 5's figure-error model)."""
        self.g = geometry
        self.n = int(n)
        self.comm = comm or LocalComm()
        self.shard = shard or Shard(0, self.n * self.n)
        if self.comm.world > 1:
            want = Shard.split(self.n, self.comm.world, self.comm.rank)
            if self.shard != want:
                raise ValueError(f"rank {self.comm.rank}'s shard must be Shard.split's {want} (buffer-aligned)")
            self._nbufs = [Shard.split(self.n, self.comm.world, r).full_buffers() for r in range(self.comm.world)]
        self.resample_pass = resample_pass
        self.dev = D.device()
        self.rand_h = geometry.angle_h.table(self.n)
        self.rand_v = geometry.angle_v.table(self.n)
        self.tan_h = torch.from_numpy(np.tan(self.rand_h)).to(self.dev)
        self.tan_v = torch.from_numpy(np.tan(self.rand_v)).to(self.dev)
        self.n_local = self.shard.count
        self.sums = RowSums()
        # fused numpy-order reductions: pass 2 -> (atan_h, atan_v, det x, y, z), nanmean for the
        # arctans and plain mean for the detector (:3583-3590); tilt -> (det1 x, y, z, total1,
        # total2), all nanmean (:3626, :3633, :3674)
        # one per run slot: run k's sums finish (on their own stream) while run k+1's pass 1 and
        # pass 2 run, and pass 2 of run k+1 refills its own slot's sink meanwhile
        self._sink2 = [LeafSink(5, self.n_local, 0b00011, self.dev) for _ in range(self.NSLOTS)]
        L = _lib.lib()
        self._fin_work = [torch.empty(max(int(L.akb_finish_params_work_bytes(s.desc)) // 8 + 1, 2), dtype=D.F64,
                                      device=self.dev) for s in self._sink2]
        # per-run buffer sets ("slots", run k uses k % 4): a pipelined caller fuses run k's tilt
        # into run k+2's pass 1 and its OPD into run k+3's, so that run k's pass-2 sums and tilt
        # parameters (their own stream) finish beside run k+1's passes, off the chain of trace
        # kernels; four runs are in flight at once. Each slot holds a pass-2 and a tilt sink, the
        # det2 extent keys (uint64 bits) its OPD folds and its pupil reads, the pass-2 tables and
        # output rows, and the flag words
        NS = self.NSLOTS
        self._sink3 = [LeafSink(5, self.n_local, 0b11111, self.dev) for _ in range(NS)]
        self._ext = torch.zeros((NS, 4), dtype=torch.int64, device=self.dev)
        self._runs = 0
        self._pitch = torch.zeros(2, dtype=D.F64, device=self.dev)
        self._opd_buf = None
        self.last = {}
        self.kernel_events = None  # set to a list to time the pass-2 chain launch (bench.py)
        self.pass1_events = None  # set to a list to time the pass-1 launch (fused or not; bench.py)
        # prepared launches. The resample picks come from a prepass that traces only the rays
        # they read (akb_trace_chain_samples_f64, every rank all of them); the pick buffer ends
        # with one double-sized slot holding that prepass's flag word, so one copy brings both to
        # the host. The full pass 1 (this shard's rays, possibly fused with the previous run's
        # tilt) then runs while the host resamples; its flag word and pass 2's ([pass 1, pass 2])
        # reach the host in one 8-byte copy after pass 2, and the tilt-parameter kernel zeroes them.
        self._plan = sample_plan(self.n)
        hb, he, col = self._plan
        self._nsamp = (he - hb) + self.n
        # the picks, then four int32 flag words [pass 1, pass 2, prepass, unused]: one copy
        # brings the picks and the prepass's word; the tilt-parameter kernel keeps and clears the
        # first two, the prepass's is zeroed on its own stream ahead of each prepass
        self._x1 = torch.zeros(self._nsamp + 2, dtype=D.F64, device=self.dev)
        words = self._x1[self._nsamp:].view(torch.int32)
        self._sflag, self._words = words[2:3], words
        self._x1_host = torch.empty((2, self._nsamp + 2), dtype=D.F64, pin_memory=True)
        self._pick_buf = 0
        self._next_picks = None  # (event, host buffer) of a prepass queued for the next run
        # per run slot (a run's front returns before its pass 2 ends, so the next run must not
        # reuse them): the [pass 1, pass 2] flag words on the host and the pass-2 tables [h | v]
        self._f_host = torch.zeros((NS, 2), dtype=torch.int32, pin_memory=True)
        # the [pass 1, pass 2] trace flag words of each run slot (the tilt-parameter kernel of a
        # run keeps and clears its slot's pair, beside the next run's passes)
        self._flagw = torch.zeros((NS, 2), dtype=torch.int32, device=self.dev)
        self._tan2 = torch.empty((NS, 2 * self.n), dtype=D.F64, device=self.dev)
        self._tan2_host = torch.empty((NS, 2 * self.n), dtype=D.F64, pin_memory=True)
        self._staged = [None] * NS  # event after the pass 1 that copied a slot's host tables
        # event after the tilt-parameter kernel of the run that last used a slot (it clears the
        # slot's flag words and reads its sink): the slot's next pass 1 waits for it if needed
        self._slot_done = [None] * NS
        self._desc_key = {}  # id(ChainLaunch) -> geometry_key its descriptor holds
        self._ps = ChainLaunch(self.g.mirrors, tan_h=self.tan_h, tan_v=self.tan_v, row0=0, n_rays=self.n * self.n,
                               src=self.g.source, want=(), samples=(hb, he, col), flags=self._sflag,
                               samples_buf=self._x1[:self._nsamp])
        self._p1 = ChainLaunch(self.g.mirrors, tan_h=self.tan_h, tan_v=self.tan_v, ray0=self.shard.start,
                               n_rays=self.n_local, src=self.g.source, want=(), flags=self._flagw[0, 0:1])
        self._p2 = {}
        self._desc_key[id(self._ps)] = self._desc_key[id(self._p1)] = geometry_key(self.g)
        self._pert = perturbation.device_tables(self.n, self.n, self.dev) if perturbation is not None else None
        # event after the last queued reader of the pass-2 buffers / extent keys (a back half
        # and its pupil, possibly on another stream): the next pass 2 waits for it
        self._back_done = None
        # two streams besides the caller's, each on a hardware queue of its own (a stream sharing
        # a queue waits behind the other stream's kernels: the box gives a process 4 queues, so
        # RayWave takes 2 and leaves one for a caller's back-half stream): the picks prepass and
        # its copy to the host (beside the trace kernels, latency-bound: the next run's resample
        # waits for it), and the finishes (a fused tilt's sums, each run's pass-2 sums and tilt
        # parameters, the flag words' copy to the host), which overlap the next passes
        self._fin = torch.cuda.Stream(device=self.dev)
        # (a high-priority copy stream measured 10 % slower). With several ranks the collectives
        # run on one more stream of their own (RCCL's): the picks then share the finish stream, so
        # that the process still fits the box's four hardware queues (the picks are needed only
        # by the next run's host resample, well after the finish kernels ahead of them)
        self._copy = torch.cuda.Stream(device=self.dev) if self.comm.world == 1 else self._fin

    def _pass2_launch(self, want_rows, slot=0):
        key = (bool(want_rows), slot)
        if key not in self._p2:
            want = ("last_hit", "dir_out", "opl") + (("det", "atan") if want_rows else ())
            # each slot writes its own output rows: run k's are tilted inside run k+2's pass 1
            t2 = self._tan2[slot]
            self._p2[key] = ChainLaunch(self.g.mirrors, tan_h=t2[:self.n], tan_v=t2[self.n:],
                                        ray0=self.shard.start, n_rays=self.n_local, src=self.g.source,
                                        det_ghij=self.g.det1, want=want, sink=self._sink2[slot],
                                        flags=self._flagw[slot, 1:2], pert=self._pert)
            self._desc_key[id(self._p2[key])] = geometry_key(self.g)
        return self._p2[key]

    # -------------------------------------------------------------- per-run geometry
    def _check_geometry(self, g):
        """A run may trace another system than the one RayWave was built for (auto_focus-style
        sweeps): its mirrors, detector planes and source may differ; the ray grid (angle ranges)
        and the number of detectors may not."""
        if g is self.g:
            return
        if (g.angle_h.start, g.angle_h.stop, g.angle_h.offset, g.angle_v.start, g.angle_v.stop, g.angle_v.offset) != (
                self.g.angle_h.start, self.g.angle_h.stop, self.g.angle_h.offset, self.g.angle_v.start,
                self.g.angle_v.stop, self.g.angle_v.offset):
            raise ValueError("a run's geometry must keep RayWave's ray-grid angle ranges")
        if (g.det2 is None) != (self.g.det2 is None) or len(g.mirrors) != len(self.g.mirrors):
            raise ValueError("a run's geometry must have as many mirrors and detector planes as RayWave's")

    def _use(self, launch, g):
        """Point a prepared chain launch at g's mirrors / detector / source (only when it holds
        another system: the descriptor is copied into the kernel arguments at each launch)."""
        key = geometry_key(g)
        if self._desc_key.get(id(launch)) != key:
            _fill_desc(launch.desc, g.mirrors, g.det1)
            for j in range(3):
                launch.desc.src[j] = float(g.source[j])
            self._desc_key[id(launch)] = key

    # -------------------------------------------------------------- passes
    def _queue_picks(self, g=None):
        """The picks prepass of the next run (system g) and its copy to the host, on the copy
        stream (it reads only the constant grid tables, so it runs one run ahead, beside this run's
        kernels); its host buffer alternates between runs."""
        g = g if g is not None else self.g
        x = self._x1_host[self._pick_buf]
        self._pick_buf ^= 1
        self._use(self._ps, g)
        with torch.cuda.stream(self._copy):
            self._sflag.zero_()
            _lib.check(_lib.lib().akb_trace_chain_samples_f64(self._ps.desc, D.stream_handle(self._copy)))
            x.copy_(self._x1, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._copy)
        self._next_picks = (ev, x, geometry_key(g))

    def _take_picks(self, g=None):
        """This run's picks and the prepass's flag word (waits for the prepass if still running).
        A prepass queued for another system than g (the caller did not announce g as the
        next_geometry) is dropped and redone for g."""
        g = g if g is not None else self.g
        if self._next_picks is not None and self._next_picks[2] != geometry_key(g):
            D.wait_event(self._next_picks[0])  # its host buffer is about to be reused
            self._next_picks = None
        if self._next_picks is None:
            self._queue_picks(g)
        ev, x, _ = self._next_picks
        self._next_picks = None
        D.wait_event(ev)
        hb, he, _ = self._plan
        host = x.numpy()
        nh = he - hb
        flags = int(host[self._nsamp:].view(np.int32)[0])
        return host[:nh].copy(), host[nh:self._nsamp].copy(), flags

    def _pass1(self, stream, fuse, slot, fuse_opd=None):
        """The full pass 1 (fused with fuse's tilt, and fuse_opd's OPD, when given). Its workgroup
        0 also stages this run's resampled tables from pinned host memory to the device
        (akb_chain_desc.copy_*), so pass 2 follows it with no copy or cross-stream wait."""
        d = self._p1.desc
        d.copy_src, d.copy_dst, d.copy_n = D.ptr(self._tan2_host[slot]), D.ptr(self._tan2[slot]), 2 * self.n
        d.flags = D.ptr(self._flagw[slot, 0:1])
        tev = None
        if self.pass1_events is not None:  # (on the stream the kernel runs on: the current one)
            tev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            tev[0].record()
        if fuse is None:
            self._p1.launch(stream=stream, reset_flags=False)
            ev = torch.cuda.Event()
            ev.record()
        else:
            ev = self._fused_pass1(fuse, stream, fuse_opd)  # one event after the kernel serves both
        if tev is not None:
            tev[1].record()
            self.pass1_events.append((tev[0], tev[1], fuse is not None, fuse_opd is not None))
        self._staged[slot] = ev

    def _pass2(self, want_rows=False, stream=None, slot=0):
        ev = None
        if self.kernel_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        r = self._pass2_launch(want_rows, slot).launch(stream=stream, reset_flags=False)
        if ev is not None:
            ev[1].record()
            self.kernel_events.append(ev)
        return r

    def _pass2_staged(self, tan_h2, tan_v2, g=None):
        """Exact stage-by-stage pass 2 (used only when the fused kernel raised a flag)."""
        g = g if g is not None else self.g
        from .trace import grid_dirs
        dirs = grid_dirs(tan_h2, tan_v2)
        lo = self.shard.start
        dirs = dirs[:, lo:lo + self.n_local].contiguous()
        src = torch.tensor(g.source, dtype=D.F64, device=self.dev).reshape(3, 1).expand(3, self.n_local)
        src = src.contiguous()
        hits, r4, segs = staged_chain(g.mirrors, dirs, src, with_segments=True)
        opl = segs[0]
        for s in segs[1:]:
            opl = opl + s
        if self._pert is not None:
            ph, pv = self._pert
            opl = opl + (pv.T @ ph).reshape(-1)[lo:lo + self.n_local]
        det = P.plane_ray_intersection([0] * 6 + list(g.det1), r4, hits[-1])
        atan = torch.stack([torch.atan(r4[1] / r4[0]), torch.atan(r4[2] / r4[0])])
        return hits[-1], r4, det, opl, atan

    # -------------------------------------------------------------- one run
    def run(self, opd=True, keep_rotated=False, full=False, overlap=None, geometry=None, next_geometry=None):
        """Trace and reduce; returns a RunResult of device tensors (this shard's rays) and means.
        keep_rotated: also return the tilted direction / last hit (dir_rot, pt_rot); full: also
        return DistError (detector 1), Sph, detcenter and the pre-tilt rows. The default keeps what
        griddata consumes (DistError2, Wave2, detcenter2) and reduces everything else on the fly.
        overlap: callable enqueuing independent device work (e.g. the previous step's PSF) that
        runs while the host performs the resample.

        last_hit / dir_out / opl are the pass-2 launch's own buffers: the next run overwrites
        them. A run is launch_back(launch_front()); a caller tracing several systems in a row can
        pass the previous run's launch_back as this run's overlap, so its tilt and OPD fill the
        GPU while the host resamples (bench.py does)."""
        return self.launch_back(self.launch_front(full=full, overlap=overlap, geometry=geometry,
                                                  next_geometry=next_geometry), opd=opd, keep_rotated=keep_rotated)

    def launch_front(self, full=False, overlap=None, fuse=None, fuse_opd=None, geometry=None, next_geometry=None):
        """The resample picks, pass 1, the resample (the run's one host wait, for the picks
        only), pass 2, its sums and the device tilt parameters. Returns as soon as all of it is
        queued; the trace flags are read when launch_back (or _resolve) needs them.

        The picks come from a prepass queued one run ahead (on the copy stream, beside the
        previous run's kernels); the host resamples, queues the next run's prepass, and pass 1
        stages the new tables for pass 2 itself: the trace kernels follow each other on the stream
        with nothing in between.

        fuse: the previous run's front, not yet handed to launch_back: its tilt then runs inside
        this run's pass-1 kernel (akb_chain_tilt_f64), its loads hidden behind the chain's
        arithmetic, and its tilt sums are finished beside this run's pass 2. fuse_opd: the front
        before that one (tilted inside the previous pass 1): its OPD maps are formed inside the same
        kernel (akb_chain_tilt_opd_f64), and its launch_back then only assembles the result (queue
        it in `overlap`, called once pass 1 is queued, so its pupil runs beside this run's pass 2).
        Without fuse_opd, fuse's launch_back forms the OPD itself. A fused OPD inside pass 2
        measured slower (1.005 vs 0.974 ms per bench step): its loads and registers cost the
        FP64-bound chain more than running beside it; pass 1 keeps nothing of it across the chain.

        geometry: the system this run traces (default: RayWave's own); consecutive runs may trace
        different systems - mirrors, detector planes, source - over the same ray grid, and the
        fused tilt / OPD of an earlier run keep that run's system (its front carries it).
        next_geometry: the system of the run after this one, whose picks prepass is queued here
        (default: this run's); announcing it keeps the prepass one run ahead."""
        L = _lib.lib()
        g = geometry if geometry is not None else self.g
        self._check_geometry(g)
        stream = D.stream_handle()
        slot = self._runs % self.NSLOTS
        self._runs += 1
        if fuse is not None and (fuse.tilt is not None or fuse.full or self.g.det2 is None):
            # the fused kernel writes the detector-2 rows only: full runs and single-detector
            # systems (KB) keep the tilt in their own back half
            fuse = None
        if fuse_opd is not None and (fuse is None or fuse_opd.tilt is None or fuse_opd.opd is not None
                                     or fuse_opd.fin_ev is None or any(self._flags_of(fuse_opd))):
            # needs a fused tilt to ride on, fuse_opd's own fused tilt, and clean trace flags
            # (a flagged run takes the staged path in its launch_back); its pass 2 ended two runs
            # ago, so reading its flags waits for nothing
            fuse_opd = None
        # fused optimistically: should fuse's pass 2 turn out flagged, launch_back ignores the
        # fused tilt and takes the staged path (its tables live in fuse's own slot)
        samp_h, samp_v, sflags = self._take_picks(g)
        if sflags:
            torch.cuda.synchronize()
            self._words.zero_()
            self._flagw.zero_()
            torch.cuda.synchronize()
            raise _lib.AKBError(self._pass1_error(sflags))
        if self._staged[slot] is not None:  # the pass 1 that last copied this slot's host tables
            D.wait_event(self._staged[slot])
            self._staged[slot] = None
        th = self._tan2_host[slot].numpy()
        if self.resample_pass:
            # np.arctan / np.tan stay numpy's (their SIMD kernels are what the reference runs)
            np.tan(resample_axis(np.arctan(samp_h), self.rand_h), out=th[:self.n])
            np.tan(resample_axis(np.arctan(samp_v), self.rand_v), out=th[self.n:])
        else:
            np.tan(self.rand_h, out=th[:self.n])
            np.tan(self.rand_v, out=th[self.n:])
        nxt = next_geometry if next_geometry is not None else g
        self._check_geometry(nxt)
        self._queue_picks(nxt)
        if fuse is not None and self._back_done is not None:
            # the back half queued before (its OPD / pupil; its extent keys are cleared by a
            # later tilt-parameter kernel and its tilt sink refilled by a later fused pass 1):
            # normally long done, and then no wait enters the stream
            self._wait(self._back_done)
            self._back_done = None
        if fuse_opd is not None:  # its tilt sums
            self._wait(fuse_opd.fin_ev)
        if fuse is not None:  # its tilt parameters
            self._wait(fuse.done)
        if self._slot_done[slot] is not None:  # the slot's last tilt parameters (a pipelined caller waited)
            self._wait(self._slot_done[slot])
            self._slot_done[slot] = None
        self._use(self._p1, g)
        self._pass1(stream, fuse, slot, fuse_opd)
        if fuse is not None:
            self._finish_tilt(fuse)
        if overlap is not None:
            overlap()  # e.g. an earlier run's back half, beside this run's pass 2
        tan_h2, tan_v2 = self._tan2[slot, :self.n], self._tan2[slot, self.n:]
        if self._back_done is not None and fuse is None:
            # pass 2 rewrites the buffers a queued (unfused) back half's tilt reads
            torch.cuda.current_stream().wait_event(self._back_done)
            self._back_done = None
        self._use(self._pass2_launch(full, slot), g)
        r = self._pass2(want_rows=full, stream=stream, slot=slot)
        # this run's pass-2 sums and tilt parameters on their own stream: they overlap the next
        # run's passes (the run is tilted two runs later, inside run k+2's pass 1)
        p2done = torch.cuda.Event()
        p2done.record()
        params = torch.empty(25, dtype=D.F64, device=self.dev)  # this run's own block
        with torch.cuda.stream(self._fin):
            self._fin.wait_event(p2done)
            ps = D.stream_handle(self._fin)
            flags = self._flagw[slot]
            if self.comm.world > 1:  # any rank's flag bits (OR, not a sum: bits must not carry)
                self.comm.allreduce_or(flags)
            if self.comm.world == 1:  # the sink's finish and the parameters in two small launches
                s2 = self._sink2[slot]
                _lib.check(L.akb_finish_tilt_params_f64(s2.desc, D.ptr(s2.sums), D.ptr(s2.counts), D.ptr(params),
                                                        D.ptr(self._ext[slot]), D.ptr(flags), 2,
                                                        D.ptr(self._fin_work[slot]), ps))
            else:
                sums, cnts = self._finish_sink(self._sink2[slot], ps)
                _lib.check(L.akb_tilt_params_f64(D.ptr(sums), D.ptr(cnts), D.ptr(params), D.ptr(self._ext[slot]),
                                                 D.ptr(flags), 2, ps))
            done = torch.cuda.Event()
            done.record(self._fin)
            # the flag words the parameter kernel kept (params[23:25]) to the host
            self._f_host[slot].copy_(params[23:24].view(torch.int32), non_blocking=True)
            ev2 = torch.cuda.Event()
            ev2.record(self._fin)
        self._slot_done[slot] = done
        params.record_stream(self._fin)
        return _Front(r=r, tan_h2=tan_h2, tan_v2=tan_v2, params=params, full=full, stream=stream, flag_ev=ev2,
                      done=done, slot=slot, g=g)

    def _wait(self, ev):
        """Order the current stream after ev (an event of RayWave's other streams) by waiting for it
        on the host: a pipelined caller runs ahead of the device, so the wait costs the device
        nothing, while a cross-queue wait on the device puts a barrier packet ahead of the next
        trace kernel (measured 0.810 -> 0.803 ms per step)."""
        D.wait_event(ev)

    def _flags_of(self, f):
        """f's (pass 1, pass 2) trace flag words (waits for its pass 2 if still running)."""
        if f.flags is None:
            D.wait_event(f.flag_ev)
            h = self._f_host[f.slot]
            f.flags = (int(h[0]), int(h[1]))
        return f.flags

    def _resolve(self, f):
        """f's trace flags (waits for its pass 2 if still running); a flagged pass 1 raises."""
        flags = self._flags_of(f)
        if flags[0]:  # the full pass 1 (its flag word arrives with pass 2's)
            raise _lib.AKBError(self._pass1_error(flags[0]))
        return flags

    @staticmethod
    def _pass1_error(flags):
        return (f"pass 1 raised trace flags {flags:#x} (a ray missed a mirror or a norm was zero): the "
                "reference returns all-NaN here and its interp1d resample fails on it")

    def _fused_pass1(self, f, stream, g=None):
        """This run's pass 1 and run f's tilt in one kernel (f's pass-2 buffers are still intact:
        this run's pass 2 comes after it on the same stream); with g (the run before f, tilted
        by the previous pass 1, its sums finished) also g's DistError2 / Wave2 and extent keys."""
        L = _lib.lib()
        tb = self._tilt_buffers(False, f.full, f.g)
        r = f.r
        n = self.n_local
        if g is None:
            _lib.check(L.akb_chain_tilt_f64(self._p1.desc, D.ptr(f.params), D.host_f64(f.g.det1),
                                            D.host_f64(tb["d2"]), D.ptr(r.dir_out), D.ptr(r.last_hit),
                                            D.ptr(r.opl), n, n, None, None, D.ptr(tb["det1"]),
                                            D.ptr(tb["det2_buf"]), D.ptr(tb["total1"]), D.ptr(tb["total2"]),
                                            self._sink3[f.slot].desc, stream))
        else:
            gt = g.tilt
            sums, cnts = g.fin
            opd = dict(dist_err2=torch.empty(n, dtype=D.F64, device=self.dev),
                       wave2=torch.empty(n, dtype=D.F64, device=self.dev))
            _lib.check(L.akb_chain_tilt_opd_f64(self._p1.desc, D.ptr(f.params), D.host_f64(f.g.det1),
                                                D.host_f64(tb["d2"]), D.ptr(r.dir_out), D.ptr(r.last_hit),
                                                D.ptr(r.opl), n, n, D.ptr(tb["det2_buf"]), D.ptr(tb["total2"]),
                                                self._sink3[f.slot].desc, D.ptr(gt["total2"]),
                                                D.ptr(gt["det2_buf"]), D.ptr(sums), D.ptr(cnts),
                                                D.ptr(opd["dist_err2"]), D.ptr(opd["wave2"]),
                                                D.ptr(self._ext[g.slot]), stream))
        ev = torch.cuda.Event()
        ev.record()
        f.tilt, f.tilted = tb, ev
        if g is not None:
            g.opd, g.opd_ev = opd, ev
        return ev

    def _finish_sink(self, sink, stream):
        """A fused sink's np.sum / np.nanmean sums and counts; across ranks in numpy's own order
        (LeafSink.finish_dist over the buffer-aligned shards): the same bits as one process."""
        if self.comm.world == 1:
            return sink.finish(stream)
        return sink.finish_dist(self.comm, self._nbufs, self.n * self.n, stream)

    def _finish_tilt(self, f):
        """The sums of f's fused tilt (on the finish stream, beside the next pass 2)."""
        with torch.cuda.stream(self._fin):
            self._fin.wait_event(f.tilted)
            sums, cnts = self._finish_sink(self._sink3[f.slot], self._fin)
            ev = torch.cuda.Event()
            ev.record(self._fin)
        f.fin, f.fin_ev = (sums, cnts), ev

    def launch_back(self, f, opd=True, keep_rotated=False, stream=None):
        """Tilt, detectors and OPD of a launch_front (no host wait). stream: run them on that
        stream instead of the front's - concurrently with the next launch_front's pass 1, which
        is FP64-bound while this half is HBM-bound; the next pass 2 waits for it (and for a pupil
        taken on the same stream). A front whose tilt and OPD were fused into later pass-1
        kernels only has its result assembled here."""
        if stream is None:
            if f.opd is None and f.fin_ev is not None:
                torch.cuda.current_stream().wait_event(f.fin_ev)
            if f.tilt is None and not f.done.query():  # its tilt parameters (own stream)
                torch.cuda.current_stream().wait_event(f.done)
            out = self._launch_back(f, opd, keep_rotated)
        else:
            stream.wait_event(f.opd_ev if f.opd is not None else f.tilted if f.tilt is not None else f.done)
            if f.opd is None and f.fin_ev is not None:
                stream.wait_event(f.fin_ev)
            f.params.record_stream(stream)  # allocated on the front's stream, read here
            for t in list((f.tilt or {}).values()) + list((f.opd or {}).values()):
                if isinstance(t, torch.Tensor):
                    t.record_stream(stream)
            with torch.cuda.stream(stream):
                out = self._launch_back(dataclasses.replace(f, stream=None), opd, keep_rotated)
        ev = torch.cuda.Event()
        ev.record(stream if stream is not None else torch.cuda.current_stream())
        self._back_done = ev
        return out

    def _launch_back(self, f, opd, keep_rotated):
        r = f.r
        if self._resolve(f)[1]:  # a flagged pass 2: the staged path (a fused tilt is discarded)
            out = self._run_staged(None, f.tan_h2, f.tan_v2, opd, keep_rotated, f.full, slot=f.slot, g=f.g)
        else:
            out = RunResult(last_hit=r.last_hit, dir_out=r.dir_out, opl=r.opl, tan_h2=f.tan_h2, tan_v2=f.tan_v2,
                            params=f.params)
            if f.full:
                out.update(det_pre=r.det, atan=r.atan)
            if f.opd is not None:  # tilted and OPD-formed inside the two next runs' pass 1
                tb = f.tilt
                self._means5 = f.fin
                out.update(dir_rot=None, pt_rot=None, detcenter=None, detcenter2=tb["det2"], total=None,
                           total2=tb["total2"], dist_err=None, sph=None, **f.opd)
            elif f.tilt is not None:  # tilted inside the next run's pass 1
                out.update(self._opd_after_tilt(f.tilt, f.full, True, f.slot, f.stream, fin=f.fin))
            elif opd:
                out.update(self._tilt_opd(r.last_hit, r.dir_out, r.opl, keep_rotated, f.full, params=f.params,
                                          stream=f.stream, slot=f.slot, g=f.g))
        out["flags"] = f.flags
        out["slot"] = f.slot
        self.last = out
        return out

    def _run_staged(self, fast, tan_h2, tan_v2, opd, keep_rotated, full, slot=0, g=None):
        """Pass 2 flagged a miss or a zero norm: redo it stage by stage (the reference's value
        rules) and the tilt from host-formed matrices."""
        torch.cuda.synchronize()
        last_hit, dir_out, det_pre, opl, atan = self._pass2_staged(tan_h2.clone(), tan_v2.clone(), g)
        (atan_s, atan_c), (det_s, det_c) = self.sums(atan, nan=True), self.sums(det_pre)
        red = self.comm.allreduce_sums(torch.cat([atan_s, det_s, atan_c.to(D.F64), det_c.to(D.F64)]))
        host = red.cpu().numpy()
        with np.errstate(invalid="ignore", divide="ignore"):
            mean_atan = host[0:2] / host[5:7]
            focus = host[2:5] / host[7:10]
        theta_y = -mean_atan[1]
        theta_z = mean_atan[0]
        out = RunResult(last_hit=last_hit, dir_out=dir_out, opl=opl, theta_y=theta_y, theta_z=theta_z,
                        focus_apprx=focus, tan_h2=tan_h2, tan_v2=tan_v2)
        if full:
            out.update(det_pre=det_pre, atan=atan)
        if opd:
            ry, rz = P.rotation_matrices(-theta_y, -theta_z)
            out.update(self._tilt_opd(last_hit, dir_out, opl, keep_rotated, full, host_tilt=(ry, rz, focus), slot=slot,
                                      g=g))
        return out

    def _tilt_buffers(self, keep_rotated, full, g=None):
        """Output tensors of one tilt (allocated on the current stream)."""
        g = g if g is not None else self.g
        n, dev = self.n_local, self.dev
        two = g.det2 is not None
        e = lambda *shape: torch.empty(shape, dtype=D.F64, device=dev)
        tb = dict(two=two, d2=g.det2 if two else g.det1,
                  det1=e(3, n) if (full or not two) else None, det2=e(3, n) if two else None,
                  total1=e(n) if (full or not two) else None, total2=e(n),
                  dir_rot=e(3, n) if keep_rotated else None, pt_rot=e(3, n) if keep_rotated else None)
        tb["det2_buf"] = tb["det2"] if two else e(3, n)
        return tb

    def _tilt_opd(self, last_hit, dir_out, opl, keep_rotated=False, full=False, host_tilt=None, params=None,
                  stream=None, slot=0, g=None):
        L = _lib.lib()
        g = g if g is not None else self.g
        n = self.n_local
        sh = D.stream_handle(stream)
        tb = self._tilt_buffers(keep_rotated, full, g)
        outs = (D.ptr(dir_out), D.ptr(last_hit), D.ptr(opl), n, n, D.ptr(tb["dir_rot"]), D.ptr(tb["pt_rot"]),
                D.ptr(tb["det1"]), D.ptr(tb["det2_buf"]), D.ptr(tb["total1"]), D.ptr(tb["total2"]),
                self._sink3[slot].desc,
                sh)
        if host_tilt is None:
            _lib.check(L.akb_tilt_opd_dev_f64(D.ptr(params), D.host_f64(g.det1), D.host_f64(tb["d2"]), *outs))
        else:
            ry, rz, focus = host_tilt
            _lib.check(L.akb_tilt_opd_f64(D.host_f64(ry.ravel()), D.host_f64(rz.ravel()), D.host_f64(focus),
                                          D.host_f64(g.det1), D.host_f64(tb["d2"]), *outs))
        return self._opd_after_tilt(tb, full, host_tilt is None, slot, stream)

    def _opd_after_tilt(self, tb, full, keys_zeroed, slot, stream, fin=None):
        """The tilt sink's means (fin: already finished), then DistError / Sph / Wave2 and the
        pupil extent keys."""
        L = _lib.lib()
        n, dev = self.n_local, self.dev
        sh = D.stream_handle(stream)
        if fin is not None:
            sums, cnts = fin
        else:
            sums, cnts = self._finish_sink(self._sink3[slot], sh)
        self._means5 = (sums, cnts)
        total1 = tb["total1"]
        dist_err = torch.empty(n, dtype=D.F64, device=dev) if total1 is not None else None
        dist_err2 = torch.empty(n, dtype=D.F64, device=dev)
        sph = torch.empty(n, dtype=D.F64, device=dev) if full else None
        wave2 = torch.empty(n, dtype=D.F64, device=dev) if tb["two"] else None
        _lib.check(L.akb_opd_f64(D.ptr(total1), D.ptr(tb["total2"]), D.ptr(tb["det2_buf"]), n, n, D.ptr(sums),
                                 D.ptr(cnts), D.ptr(dist_err), D.ptr(dist_err2), D.ptr(sph), D.ptr(wave2),
                                 D.ptr(self._ext[slot]), int(bool(keys_zeroed)), sh))
        return dict(dir_rot=tb["dir_rot"], pt_rot=tb["pt_rot"], detcenter=tb["det1"], detcenter2=tb["det2"],
                    total=total1, total2=tb["total2"], dist_err=dist_err, dist_err2=dist_err2, sph=sph, wave2=wave2)

    def means(self):
        """Host copies of the post-tilt means: (mean_total [detector 1, detector 2], mean_focus)."""
        s, c = self._means5
        h = torch.cat([s, c.to(D.F64)]).cpu().numpy()
        m = h[:5] / h[5:]
        return m[3:5], m[0:3]

    # -------------------------------------------------------------- pupil for the PSF
    def pupil(self, size=128):
        """Wave2 (nm) sampled onto a size x size pupil in ray-index space (nearest ray), as OPD in
        metres, and the pupil pitch of the detector-2 footprint (device [dx, dy]).

        A fast stand-in for griddata(cubic) + plane correction + rotate_with_nan of the driver
        (:3689-3710, psf_calc :1121-1188), used by the bench's PSF: the ray grid is a smooth
        deformed structured grid, so index-space sampling keeps the pupil's shape. The faithful
        chain is pupilmap.wave_maps + psfcalc.psf_calc. The amplitude is
        psf_calc's mask (1 where the OPD is defined), formed inside the PSF kernel.
        Multi-GPU: each shard fills its rows and the pieces are summed over ranks."""
        L = _lib.lib()
        if self._opd_buf is None or self._opd_buf.shape[0] != size:
            self._opd_buf = torch.empty((size, size), dtype=D.F64, device=self.dev)
        ext = self._ext[self.last.get("slot", 0)]
        if self.comm.world > 1:
            # unsigned key order == signed order after flipping the top bit: MAX over ranks
            # (a Python-int operand: no host-to-device copy of a constant, which would wait for the stream)
            flip = -(1 << 63)
            ext = self.comm.allreduce_max(torch.bitwise_xor(ext, flip)).bitwise_xor(flip).contiguous()
        _lib.check(L.akb_pupil_sample_f64(D.ptr(self.last["wave2"]), self.shard.start, self.shard.count, self.n,
                                          size, D.ptr(ext), D.ptr(self._opd_buf), D.ptr(self._pitch),
                                          D.stream_handle()))
        opd = self._opd_buf
        if self.comm.world > 1:
            opd = self.comm.allreduce_sums(opd)
        ev = torch.cuda.Event()
        ev.record()
        self._back_done = ev  # reads the extent keys the next tilt-parameter kernel clears
        return opd, self._pitch

    # -------------------------------------------------------------- accounting
    def intersections_per_run(self):
        """Ray-surface intersections computed per run by this shard: 2 passes x K mirrors."""
        return 2 * len(self.g.mirrors) * self.n_local
