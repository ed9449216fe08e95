"""The reference's own PSF of a traced run, pipelined on the device.

plot_result_debug's 'ray_wave' step after the trace (AKB_raytrace_20250312.py:3653-3700):

    grid_H, grid_V = meshgrid(linspace(min, max) of detcenter2[1], [2])        :3654-3657
    matrixWave2 = griddata((y, z), Wave2, (grid_H, grid_V), 'cubic')            :3689
    matrixWave2 -= nanmean(matrixWave2);  plane_correction_...(matrixWave2)     :3690, :3693
    psf_calc(matrixWave2_Corrected, grid_H, grid_V, defocusWave)                :3698-3700

FaithfulPupil runs it for run after run without a host wait on the queuing thread:

  begin(y, z)   on the caller's stream: the boundary ring (akb_gd_ring_f64), the target axes from
                it (akb_gd_axes_f64), the cell diagonals and checks with the cells' target claims
                fused in (akb_gd_cells_claims_f64), the ring and the cell flags to pinned host memory
                in one copy; a worker thread then checks the flags and builds the hull pockets
                (akb_gd_pockets, host C++ - the only host step, off the GIL);
  finish(t, f)  once that ticket's pockets are built: the pocket arrays to the device, their
                local-Delaunay check and target claims (akb_gd_claim_pockets_f64), griddata by the
                cone solve (akb_gd_cone_solve_f64: CONE_SWEEPS Chebyshev sweeps formed only where
                the targets read them, the Clough-Tocher patches), the nanmean removal,
                plane correction, rotation estimate and rotate_with_nan in one workgroup
                (akb_pupil_post_f64), and the pad-16 PSF (akb_psf_f64). All on the stream, no host
                synchronisation; errors the reference would raise surface in Ticket.check().

The host-synchronous drop-ins (griddata.griddata, pupilmap.wave_pupil, psfcalc.psf_calc) stay the
API for single calls; tests/test_faithful_gpu.py holds this pipeline to them and to the
reference's own PSF.
"""
import concurrent.futures
import time

import numpy as np
import torch

from . import _lib
from . import device as D
from .griddata import CONE_GUARD, CONE_SWEEPS, _F_NEG, _F_NONCONVEX, _F_NONFINITE, _F_NOT_DELAUNAY, _F_POCKET, _F_POS
from .griddata import ConeNotConverged, CubicGrid, chebyshev_weights
from .psf import psf_stack
from .pupilmap import POST_PARAMS, pupil_post, pupil_post_check

EUV = 13.5e-9  # option_energy 'EUV' (:1161-1162)


def pack_pockets(buf, o, Lr):
    """Pack a pocket block (akb_gd_pockets' arrays at their capacity offsets o) in place so that
    what the device reads is one prefix: tri (3 npk) | nbr (3 npk) | edge (L) | xptr (L + 1) | xidx
    (xptr[L]). Returns (npk, the packed offsets with their total length under "len"); the H2D copy
    is then that prefix (~half the capacity block at C3) instead of the whole block."""
    npk = int(buf[o["npk"]])
    nx = int(buf[o["xptr"] + Lr])
    nbr = buf[o["nbr"]:o["nbr"] + 3 * npk].copy()
    rest = np.concatenate([buf[o["edge"]:o["edge"] + Lr], buf[o["xptr"]:o["xptr"] + Lr + 1],
                           buf[o["xidx"]:o["xidx"] + nx]])
    p = dict(tri=0, nbr=3 * npk, edge=6 * npk, xptr=6 * npk + Lr, xidx=6 * npk + 2 * Lr + 1)
    assert o["tri"] == 0
    buf[p["nbr"]:p["nbr"] + 3 * npk] = nbr
    buf[p["edge"]:p["edge"] + rest.size] = rest
    p["len"] = p["edge"] + rest.size
    return npk, p


class ErrorLog:
    """Each finished run's error words, copied device -> pinned host memory at the end of its finish
    (stream-ordered: no wait on the queuing thread), one row per run. A ticket's check() then reads
    its own run's words however many runs later it is called - the device buffers they come from
    (FaithfulPupil.words: the status word, the change and estimate, the post parameters) are
    rewritten by every later finish.
    Rows are reused after `cap` finishes; a ticket whose row was reused refuses to report."""

    def __init__(self, width, cap=8192):
        self.buf = torch.zeros((int(cap), int(width)), dtype=D.F64, pin_memory=True)
        self.seq = np.full(int(cap), -1, dtype=np.int64)
        self.count = 0

    def record(self, parts, stream):
        """Queue the copies of `parts` (float64 device tensors, or int64 ones viewed as float64 bits)
        into the next row on `stream`. Returns (row, sequence number)."""
        r = self.count % self.buf.shape[0]
        seq = self.count
        self.seq[r] = seq
        self.count += 1
        off = 0
        with torch.cuda.stream(stream):
            for t in parts:
                k = t.numel()
                self.buf[r, off:off + k].copy_(t.reshape(-1), non_blocking=True)
                off += k
        return r, seq

    def read(self, row, seq, done):
        """The row's words once `done` (the run's end event) has passed."""
        if self.seq[row] != seq:
            raise RuntimeError(f"the error words of run {seq} were overwritten ({self.buf.shape[0]} runs later)")
        done.synchronize()
        return self.buf[row].numpy().copy()


class Ticket:
    """One run in the pipeline: its slot, the tensors it reads, the pocket job, then its results."""

    __slots__ = ("slot", "y", "z", "f", "job", "npock", "result", "h2d", "finished", "done", "log", "erow")

    def ready(self):
        return self.job.done()

    def check(self):
        """Raise as the host chain would (waits for the device): non-finite hits, a lattice that is
        not a convex unfolded grid, pockets that are not locally Delaunay, too few points for the
        plane fits. Reads this run's own error words (ErrorLog), not the slot's current ones."""
        self.job.result()
        if self.erow is None:  # begun, never finished: the pocket job's checks are all there is
            return
        w = self.log.read(*self.erow, self.done)
        st = int(w[:1].view(np.int64)[0])
        if st & (_F_NOT_DELAUNAY | _F_POCKET):
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
        pupil_post_check(w[3:])
        cone_guard(w[2], w[3:])


def cone_guard(est, params):
    """Raise ConeNotConverged when the cone solve's value-error estimate - interior targets
    (k_gd_cone_patch): 2 sqrt2 x the corners' one-more-sweep step x the cell's longest side; band
    and pocket targets (k_gd_eval): twice the value change one more sweep makes there - exceeds
    CONE_GUARD of the gridded map's range (the post block's nanmin / nanmax)."""
    rng = float(params[19]) - float(params[18])
    if not (est <= CONE_GUARD * rng):
        raise ConeNotConverged(f"griddata: the cone solve's {CONE_SWEEPS}-sweep gradients leave a value error "
                               f"estimate of {est:.3g} ({est / rng if rng > 0 else float('nan'):.2e} of the map's "
                               f"range, bar {CONE_GUARD:g}); re-run with the converged gradients")


class FaithfulPupil:
    """The faithful pupil and PSF of runs traced on an n_v x n_h ray grid (see the module doc).
    size: the pupil grid (the bench's 128); pad: psf_calc's pad factor (16); slots: runs between
    begin and finish; workers: pocket builders running at once."""

    def __init__(self, n_v, n_h, size=128, pad=16, wavelengths=(EUV,), sweeps=CONE_SWEEPS, slots=6, workers=4,
                 delaunay_tol=1e-10):
        L = _lib.lib()
        self.dev = D.device()
        self.nv, self.nh = int(n_v), int(n_h)
        self.size, self.pad, self.sweeps = int(size), int(pad), int(sweeps)
        self.lams = [float(w) for w in wavelengths]
        self.tol = float(delaunay_tol)
        self.L = 2 * (self.nh - 1) + 2 * (self.nv - 1)
        nc = (self.nv - 1) * (self.nh - 1)
        Lr = self.L
        cap = Lr
        # pocket arrays in one int32 block: tri (3 cap) | nbr (3 cap) | edge (L) | xptr (L + 1) | xidx (6 cap) | npk
        self._o = dict(tri=0, nbr=3 * cap, edge=6 * cap, xptr=6 * cap + Lr, xidx=6 * cap + 2 * Lr + 1)
        self._o["npk"] = self._o["xidx"] + 6 * cap
        self._pk_len = self._o["npk"] + 1
        self.slots = []
        for _ in range(int(slots)):
            self.slots.append(dict(
                diag=torch.empty(nc, dtype=torch.uint8, device=self.dev),
                ring=torch.zeros(2 * Lr + 1, dtype=D.F64, device=self.dev),
                ring_host=torch.empty(2 * Lr + 1, dtype=D.F64, pin_memory=True),
                pk_host=torch.zeros(self._pk_len, dtype=torch.int32, pin_memory=True),
                pk=torch.zeros(self._pk_len, dtype=torch.int32, device=self.dev),
                owner=torch.empty(self.size * self.size, dtype=torch.int32, device=self.dev),
                axes=torch.empty(2 * self.size + 6, dtype=D.F64, device=self.dev),  # gx | gy | extent | pitch
                last=None))
        self._next = 0
        m = self.size * self.size
        self.work = torch.empty(int(L.akb_gd_cone_work_bytes(self.nv, self.nh, self.size, self.size, 1)) // 8 + 1,
                                dtype=D.F64, device=self.dev)
        self.map = torch.empty((1, self.size, self.size), dtype=D.F64, device=self.dev)
        # a finish's error words in one block, copied to the ErrorLog in one transfer: the pocket
        # status word (int64 bits) | the cone's change measure and value-error estimate (ordered
        # double bits) | pupil_post's parameter block
        self.words = torch.zeros(1 + 2 + POST_PARAMS, dtype=D.F64, device=self.dev)
        self.status = self.words[:1].view(torch.int64)
        self.change = self.words[1:3].view(torch.int64)
        self.post = {"params": self.words[3:]}
        self.psf = None
        self._done = None  # the latest finish's end (finishes share work / map / pupil / psf buffers)
        self._omegas = D.host_f64(chebyshev_weights(max(self.sweeps, 1)))
        self.pool = concurrent.futures.ThreadPoolExecutor(max_workers=int(workers), thread_name_prefix="akb-pockets")
        # per run: the pocket status word (int64 bits) | the cone's change and error estimate | the post
        # parameter block
        self.errors = ErrorLog(1 + 2 + POST_PARAMS)
        self.finished = 0  # runs through finish()
        self.pocket_ms = []  # host time of each run's pocket triangulation (worker threads)

    # ------------------------------------------------------------------ stage 1
    def begin(self, y, z, f, stream=None):
        """Queue the cell pass of one run's detector hits (y, z: (n,) device rows, e.g. detcenter2[1],
        [2]; f: its Wave2) on `stream` and start its pocket job. Returns a Ticket."""
        L = _lib.lib()
        s = self.slots[self._next]
        self._next = (self._next + 1) % len(self.slots)
        if s["last"] is not None:  # the slot's previous run must be through its finish (pinned buffers)
            prev = s["last"]
            if not prev.finished:
                raise RuntimeError("FaithfulPupil: more runs begun than slots before a finish")
            if prev.h2d is not None:
                D.wait_event(prev.h2d)
        sh = D.stream_handle(stream)
        Lr = self.L
        ring = s["ring"]
        flags = ring.view(torch.int32)[4 * Lr:4 * Lr + 1]
        st = torch.cuda.current_stream() if stream is None else stream
        if s["last"] is not None and s["last"].done is not None:  # the slot's last reader, on any stream
            st.wait_event(s["last"].done)
        for a in (y, z, f):  # read on this stream now and in finish: not to be reused before
            a.record_stream(st)
        m = self.size
        gx, gy = s["axes"][:m], s["axes"][m:2 * m]
        with torch.cuda.stream(st):
            flags.zero_()
            _lib.check(L.akb_gd_ring_f64(D.ptr(y), D.ptr(z), self.nv, self.nh, D.ptr(ring[:Lr]), D.ptr(ring[Lr:2 * Lr]),
                                         D.ptr(flags), sh))
            _lib.check(L.akb_gd_axes_f64(D.ptr(ring[:Lr]), D.ptr(ring[Lr:2 * Lr]), Lr, m, m, D.ptr(gx), D.ptr(gy),
                                         D.ptr(s["axes"][2 * m:]), sh))
            _lib.check(L.akb_gd_cells_claims_f64(D.ptr(y), D.ptr(z), self.nv, self.nh, D.ptr(s["diag"]), self.tol,
                                                 D.ptr(flags), D.ptr(gx), m, D.ptr(gy), m, D.ptr(s["owner"]), sh))
            s["ring_host"].copy_(ring, non_blocking=True)  # the ring and the cell flags, one copy
            ev = torch.cuda.Event()
            ev.record(st)
        t = Ticket()
        t.slot, t.y, t.z, t.f = s, y, z, f
        t.npock, t.result, t.h2d, t.finished, t.done, t.log, t.erow = None, None, None, False, None, self.errors, None
        t.job = self.pool.submit(self._pockets, s, ev)
        s["last"] = t
        return t

    def _pockets(self, s, ev):
        """Worker thread: wait for the ring and the cell flags on the host, build the pockets, check
        the flags - their errors first, as the host chain raises them."""
        ev.synchronize()
        L = _lib.lib()
        Lr = self.L
        rb = s["ring_host"].numpy()
        err, npk = None, None
        if np.isfinite(rb[:2 * Lr]).all():
            buf = s["pk_host"].numpy()
            o = self._o
            hp = lambda k: buf[o[k]:].ctypes.data_as(_lib.c_vp)  # noqa: E731
            try:
                t0 = time.perf_counter()
                _lib.check(L.akb_gd_pockets(rb[:Lr].ctypes.data_as(_lib.c_vp), rb[Lr:2 * Lr].ctypes.data_as(_lib.c_vp),
                                            self.nv, self.nh, Lr, hp("npk"), hp("tri"), hp("nbr"), hp("edge"),
                                            hp("xptr"), hp("xidx")))
                npk, s["po"] = pack_pockets(buf, o, Lr)
                self.pocket_ms.append((time.perf_counter() - t0) * 1e3)  # (the host's pocket job, bench.py)
            except _lib.AKBError as e:
                err = e
        fl = int(rb[2 * Lr:].view(np.int32)[0])
        if fl & _F_NONFINITE:
            raise ValueError("griddata: non-finite point coordinates (a ray that missed)")
        if fl & _F_NONCONVEX or (fl & _F_POS and fl & _F_NEG):
            raise _lib.AKBError("griddata: the points do not form a convex, unfolded lattice")
        if fl & _F_NOT_DELAUNAY:
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
        if err is not None:
            raise err
        return npk

    # ------------------------------------------------------------------ stage 2
    def finish(self, t, stream=None, events=None, psf_events=None, post_events=None):
        """Queue the rest of ticket t's chain on `stream` (waits for its pocket job on the host -
        normally long done). Returns dict(psf (B, P, P) device, map, corrected, rotated, params,
        axes, change); the buffers are reused by the next finish on the stream (axes, the slot's, by
        the slot's next begin). events: optional (start, end)
        timing events recorded around the device work; psf_events: the same around the PSF alone;
        post_events: around the post (nanmean, plane fits, prefilter, rotation)."""
        L = _lib.lib()
        try:
            t.npock = D.wait_result(t.job)
        except BaseException:
            # the run failed on the host (check() raises it again); its slot stays usable
            t.y = t.z = t.f = None
            t.finished = True
            raise
        s = t.slot
        st = torch.cuda.current_stream() if stream is None else stream
        sh = D.stream_handle(st)
        o, Lr = s["po"], self.L
        with torch.cuda.stream(st):
            if self._done is not None:  # the shared buffers' last finish, on any stream
                st.wait_event(self._done)
            if events is not None:
                events[0].record(st)
            s["pk"][:o["len"]].copy_(s["pk_host"][:o["len"]], non_blocking=True)
            t.h2d = torch.cuda.Event()
            t.h2d.record(st)
            pk = s["pk"]
            k = max(t.npock, 1)
            ptri, pnbr = pk[o["tri"]:o["tri"] + 3 * k], pk[o["nbr"]:o["nbr"] + 3 * k]
            edge, xptr, xidx = pk[o["edge"]:o["edge"] + Lr], pk[o["xptr"]:o["xptr"] + Lr + 1], pk[o["xidx"]:o["len"] + 1]
            tri = (D.ptr(t.y), D.ptr(t.z), self.nv, self.nh, D.ptr(s["diag"]), t.npock, D.ptr(ptri), D.ptr(pnbr),
                   D.ptr(edge))
            self.words[:3].zero_()  # the status word, change and estimate
            _lib.check(L.akb_gd_check_pockets(*tri, self.tol, D.ptr(self.status), sh))
            m = self.size
            axes = s["axes"]
            gx, gy = axes[:m], axes[m:2 * m]
            _lib.check(L.akb_gd_claim_pockets_f64(D.ptr(t.y), D.ptr(t.z), self.nv, self.nh, D.ptr(s["diag"]), t.npock,
                                                  D.ptr(ptri), D.ptr(gx), m, D.ptr(gy), m, D.ptr(s["owner"]), sh))
            _lib.check(L.akb_gd_cone_solve_f64(*tri, D.ptr(xptr), D.ptr(xidx), D.ptr(gx), m, D.ptr(gy), m,
                                               D.ptr(t.f), 1, self.sweeps, self._omegas, D.ptr(self.work),
                                               D.ptr(s["owner"]), D.ptr(self.map), D.ptr(self.change), sh))
            if post_events is not None:
                post_events[0].record(st)
            post = pupil_post(self.map[0], out=self.post, stream=st)
            if post_events is not None:
                post_events[1].record(st)
            self.post = post
            if psf_events is not None:
                psf_events[0].record(st)
            psf, _, _ = psf_stack(post["opd"], None, self.lams, None, pad_factor=self.pad, stream=st, out=self.psf,
                                  pitch=axes[2 * m + 4:2 * m + 6])
            if psf_events is not None:
                psf_events[1].record(st)
            self.psf = psf
            if events is not None:
                events[1].record(st)
            t.erow = self.errors.record((self.words,), st)
            t.done = torch.cuda.Event()
            t.done.record(st)
            self._done = t.done
        t.result = dict(psf=psf, map=self.map[0], corrected=post["corrected"], rotated=post["rotated"],
                        params=post["params"], axes=axes, change=self.change)
        t.y = t.z = t.f = None
        t.finished = True
        self.finished += 1
        return t.result

    def run(self, y, z, f, stream=None):
        """begin + finish + check of one run (the pocket job waited for at once). A run whose cone
        solve fails its guard (ConeNotConverged) is formed again from the converged gradients
        (CubicGrid.interp: the global sweeps to scipy's tolerance) on the same axes."""
        t = self.begin(y, z, f, stream)
        r = self.finish(t, stream)
        try:
            t.check()
        except ConeNotConverged:
            r = self._converged(y, z, f, t.slot["axes"], stream)
        return r

    def _converged(self, y, z, f, ax, stream=None):
        """The run's map from the global gradient iteration (host-synchronous) on the run's axes ax,
        then the same post and PSF on the device; the result in finish's buffers."""
        st = torch.cuda.current_stream() if stream is None else stream
        m = self.size
        with torch.cuda.stream(st):
            cg = CubicGrid(y, z, self.nv, self.nh, delaunay_tol=self.tol)
            self.map[0].copy_(cg.interp(f.reshape(1, -1), ax[:m], ax[m:2 * m])[0])
            post = pupil_post(self.map[0], out=self.post, stream=st)
            self.post = post
            psf, _, _ = psf_stack(post["opd"], None, self.lams, None, pad_factor=self.pad, stream=st, out=self.psf,
                                  pitch=ax[2 * m + 4:2 * m + 6])
            self.psf = psf
            # the shared map / post / psf buffers' last writer: a later finish on another stream waits
            # for this one, not for the run's own (earlier) finish
            self._done = torch.cuda.Event()
            self._done.record(st)
        pupil_post_check(post["params"])
        return dict(psf=psf, map=self.map[0], corrected=post["corrected"], rotated=post["rotated"],
                    params=post["params"], axes=ax, change=self.change, converged=True)

    def close(self):
        self.pool.shutdown(wait=True)


def image_axes_of(result, pad=16, wavelength=EUV, defocus=1e-2):
    """x_im, y_im of psf_calc for a finished result (host): the pupil pitch after the driver's
    grid_H -= mean (:3698) from the device axes."""
    from .psf import image_axes
    a = result["axes"].cpu().numpy()
    m = (a.size - 6) // 2
    gh, gv = np.meshgrid(a[:m], a[m:2 * m])
    gh, gv = gh - np.mean(gh), gv - np.mean(gv)
    dx, dy = np.abs(gh[0, 1] - gh[0, 0]), np.abs(gv[1, 0] - gv[0, 0])
    return image_axes(m * pad, m * pad, dx, dy, wavelength, defocus)
