"""The wavefront hot path of the AKB / KB drivers, device-resident.

One call of RayWave.run() is what plot_result_debug(params, 'ray_wave') does between setting up
its mirrors and calling griddata (AKB_raytrace_20250312.py:2675-3689), on an n x n ray grid:

  pass 1    fused chain over the grid, exit slopes of the middle row/column     :2770-2845
  resample  np.arctan + scipy interp1d on the host (2n values)                  :2849-2879
  pass 2    fused chain + OPL + pre-tilt detector + arctan of the exit slopes   :2881-2905
  means     numpy-exact device sums -> theta_y, theta_z, focus_apprx            :3583-3591
  tilt      rotate direction / last hit (dgemm FMA order), detectors 1 and 2,
            totalDist, totalDist2                                               :3592-3633
  OPD       DistError2, Sph, Wave2 = DistError2 - Sph                           :3626-3677

The same object serves KB_debug (2 mirrors, :10948-11054) and any quadric chain. Geometry is
a SystemGeometry: the mirrors in trace order, detector planes and the ray-grid angle ranges.
Multi-GPU: pass a Shard (contiguous V-rows of the grid) and a communicator (see dist.py); the
only exchanges are the 2n resample samples, a handful of means and the flag word.
"""
import json
from dataclasses import dataclass, field

import numpy as np
import torch
from scipy.interpolate import interp1d

from . import _lib
from . import device as D
from . import primitives as P
from .reduce import RowSums, means_to_host
from .trace import Mirror, staged_chain, trace_chain


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


@dataclass
class Shard:
    """Contiguous block of V-rows [row0, row0 + rows) of the n x n ray grid."""
    row0: int
    rows: int

    @staticmethod
    def split(n, world, rank):
        base, rem = divmod(n, world)
        rows = base + (1 if rank < rem else 0)
        row0 = rank * base + min(rank, rem)
        return Shard(row0, rows)


def sample_plan(n):
    """Indices of the equal-angle resample picks (:2851-2856): column round((n-1)/2) and the flat
    range [round(n(n-1)/2), round(n(n+1)/2))."""
    col = round((n - 1) / 2)
    return round(n * (n - 1) / 2), round(n * (n + 1) / 2), col


def sample_ownership(shard, n):
    """Which resample picks a shard's rays supply: (mask over the middle-row range, mask over the
    n rows of the middle column)."""
    hb, he, _ = sample_plan(n)
    lo, hi = shard.row0 * n, (shard.row0 + shard.rows) * n
    own_h = np.zeros(he - hb, dtype=bool)
    own_h[max(lo, hb) - hb:max(min(hi, he) - hb, 0)] = True
    own_v = np.zeros(n, dtype=bool)
    own_v[shard.row0:shard.row0 + shard.rows] = True
    return own_h, own_v


def resample(angle_h_sep, angle_v_sep, rand_h, rand_v):
    """:2861-2870 — interp1d of the launch angles onto equally spaced exit angles."""
    out_v = np.linspace(angle_v_sep[0], angle_v_sep[-1], len(angle_v_sep))
    out_h = np.linspace(angle_h_sep[0], angle_h_sep[-1], len(angle_h_sep))
    new_v = interp1d(angle_v_sep, rand_v, kind="linear")(out_v)
    new_h = interp1d(angle_h_sep, rand_h, kind="linear")(out_h)
    return new_h, new_v


class LocalComm:
    """Single-process communicator (world of one)."""
    world = 1
    rank = 0

    def gather_samples(self, samp_h, samp_v, shard, n):
        return samp_h, samp_v

    def sum_flags(self, f):
        return f

    def allreduce_sums(self, t):
        return t

    def allreduce_max(self, t):
        return t


class RayWave:
    """Device-resident 'ray_wave' / 'wave' trace on an n x n grid (one shard of it)."""

    def __init__(self, geometry, n, shard=None, comm=None, resample_pass=True):
        self.g = geometry
        self.n = int(n)
        self.comm = comm or LocalComm()
        self.shard = shard or Shard(0, self.n)
        self.resample_pass = resample_pass
        self.dev = D.device()
        self.rand_h = geometry.angle_h.table(self.n)
        self.rand_v = geometry.angle_v.table(self.n)
        self.tan_h = torch.from_numpy(np.tan(self.rand_h)).to(self.dev)
        self.tan_v = torch.from_numpy(np.tan(self.rand_v)).to(self.dev)
        self.n_local = self.shard.rows * self.n
        self.sums = RowSums()
        self._buf1, self._buf2 = {}, {}
        self.last = {}
        self.kernel_events = None  # set to a list to time the pass-2 chain launch (bench.py)

    # -------------------------------------------------------------- passes
    def _pass1(self):
        hb, he, col = sample_plan(self.n)
        r = trace_chain(self.g.mirrors, tan_h=self.tan_h, tan_v=self.tan_v, row0=self.shard.row0,
                        n_rays=self.n_local, src=self.g.source, want=(), samples=(hb, he, col),
                        out=self._buf1)
        self._buf1 = r.extra["buffers"]
        # this shard's pieces of the picks; NaN where another shard owns them
        sh = r.samp_h
        sv = r.samp_v
        host = torch.cat([sh, sv, r.flags.to(D.F64)]).cpu().numpy()
        samp_h = host[:he - hb]
        samp_v = host[he - hb:he - hb + self.n]
        flags = int(host[-1])
        own_h, own_v = sample_ownership(self.shard, self.n)
        samp_h = np.where(own_h, samp_h, 0.0)
        samp_v = np.where(own_v, samp_v, 0.0)
        samp_h, samp_v = self.comm.gather_samples(samp_h, samp_v, self.shard, self.n)
        flags = self.comm.sum_flags(flags)
        return samp_h, samp_v, flags

    def _pass2(self, tan_h2, tan_v2):
        ev = None
        if self.kernel_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        r = trace_chain(self.g.mirrors, tan_h=tan_h2, tan_v=tan_v2, row0=self.shard.row0, n_rays=self.n_local,
                        src=self.g.source, det_ghij=self.g.det1,
                        want=("last_hit", "dir_out", "det", "opl", "atan"), out=self._buf2)
        if ev is not None:
            ev[1].record()
            self.kernel_events.append(ev)
        self._buf2 = r.extra["buffers"]
        return r

    def _pass2_staged(self, tan_h2, tan_v2):
        """Exact stage-by-stage pass 2 (used only when the fused kernel raised a flag)."""
        from .trace import grid_dirs
        dirs = grid_dirs(tan_h2, tan_v2)
        lo = self.shard.row0 * self.n
        dirs = dirs[:, lo:lo + self.n_local].contiguous()
        src = torch.tensor(self.g.source, dtype=D.F64, device=self.dev).reshape(3, 1).expand(3, self.n_local)
        src = src.contiguous()
        hits, r4, segs = staged_chain(self.g.mirrors, dirs, src, with_segments=True)
        opl = segs[0]
        for s in segs[1:]:
            opl = opl + s
        det = P.plane_ray_intersection([0] * 6 + list(self.g.det1), r4, hits[-1])
        atan = torch.stack([torch.atan(r4[1] / r4[0]), torch.atan(r4[2] / r4[0])])
        return hits[-1], r4, det, opl, atan

    # -------------------------------------------------------------- one run
    def run(self, opd=True, keep_rotated=False, full=False):
        """Trace and reduce; returns a dict of device tensors (this shard's rays) and host means.
        keep_rotated: also return the tilted direction / last hit (dir_rot, pt_rot); full: also
        return DistError (detector 1) and Sph. The default keeps what griddata consumes
        (DistError2, Wave2, detcenter2) plus the reduction inputs."""
        samp_h, samp_v, flags1 = self._pass1()
        if flags1:
            raise _lib.AKBError(
                f"pass 1 raised trace flags {flags1:#x} (a ray missed a mirror or a norm was zero): the "
                "reference returns all-NaN here and its interp1d resample fails on it")
        if self.resample_pass:
            new_h, new_v = resample(np.arctan(samp_h), np.arctan(samp_v), self.rand_h, self.rand_v)
        else:
            new_h, new_v = self.rand_h, self.rand_v
        tan_h2 = torch.from_numpy(np.tan(new_h)).to(self.dev)
        tan_v2 = torch.from_numpy(np.tan(new_v)).to(self.dev)
        r = self._pass2(tan_h2, tan_v2)
        atan_s, atan_c = self.sums(r.atan, nan=True)
        det_s, det_c = self.sums(r.det, nan=False)
        red = torch.cat([atan_s, det_s, atan_c.to(D.F64), det_c.to(D.F64), r.flags.to(D.F64)])
        red = self.comm.allreduce_sums(red)
        host = red.cpu().numpy()
        flags2 = int(host[-1])
        last_hit, dir_out, det, opl, atan = r.last_hit, r.dir_out, r.det, r.opl, r.atan
        if flags2:
            last_hit, dir_out, det, opl, atan = self._pass2_staged(tan_h2, tan_v2)
            (atan_s, atan_c), (det_s, det_c) = self.sums(atan, nan=True), self.sums(det)
            red = self.comm.allreduce_sums(torch.cat([atan_s, det_s, atan_c.to(D.F64), det_c.to(D.F64)]))
            host = red.cpu().numpy()
        with np.errstate(invalid="ignore", divide="ignore"):
            mean_atan = host[0:2] / host[5:7]
            focus = host[2:5] / host[7:10]
        theta_y = -mean_atan[1]
        theta_z = mean_atan[0]
        out = dict(last_hit=last_hit, dir_out=dir_out, det_pre=det, opl=opl, theta_y=theta_y, theta_z=theta_z,
                   focus_apprx=focus, tan_h2=tan_h2, tan_v2=tan_v2, flags=(flags1, flags2))
        if opd:
            out.update(self._tilt_opd(last_hit, dir_out, opl, theta_y, theta_z, focus, keep_rotated, full))
        self.last = out
        return out

    def _tilt_opd(self, last_hit, dir_out, opl, theta_y, theta_z, focus, keep_rotated=False, full=False):
        L = _lib.lib()
        n = self.n_local
        ry, rz = P.rotation_matrices(-theta_y, -theta_z)
        det1 = torch.empty((3, n), dtype=D.F64, device=self.dev)
        det2 = torch.empty((3, n), dtype=D.F64, device=self.dev) if self.g.det2 is not None else None
        totals = torch.empty((2, n), dtype=D.F64, device=self.dev)
        dir_rot = torch.empty((3, n), dtype=D.F64, device=self.dev) if keep_rotated else None
        pt_rot = torch.empty((3, n), dtype=D.F64, device=self.dev) if keep_rotated else None
        d2 = self.g.det2 if self.g.det2 is not None else self.g.det1
        _lib.check(L.akb_tilt_opd_f64(D.host_f64(ry.ravel()), D.host_f64(rz.ravel()), D.host_f64(focus),
                                      D.host_f64(self.g.det1), D.host_f64(d2), D.ptr(dir_out), D.ptr(last_hit),
                                      D.ptr(opl), n, n, D.ptr(dir_rot), D.ptr(pt_rot), D.ptr(det1),
                                      D.ptr(det2), D.ptr(totals), D.ptr(totals[1]), D.stream_handle()))
        tot_s, tot_c = self.sums(totals, nan=True)
        det_s, det_c = self.sums(det1, nan=True)
        red = self.comm.allreduce_sums(torch.cat([tot_s, det_s, tot_c.to(D.F64), det_c.to(D.F64)]))
        host = red.cpu().numpy()
        with np.errstate(invalid="ignore", divide="ignore"):
            mean_tot = host[0:2] / host[5:7]
            mean_focus = host[2:5] / host[7:10]
        dist_err = torch.empty(n, dtype=D.F64, device=self.dev) if (full or det2 is None) else None
        res = dict(dir_rot=dir_rot, pt_rot=pt_rot, detcenter=det1, detcenter2=det2, total=totals[0],
                   total2=totals[1], mean_total=mean_tot, mean_focus=mean_focus, dist_err=dist_err)
        if det2 is not None:
            dist_err2 = torch.empty(n, dtype=D.F64, device=self.dev)
            sph = torch.empty(n, dtype=D.F64, device=self.dev) if full else None
            wave2 = torch.empty(n, dtype=D.F64, device=self.dev)
            _lib.check(L.akb_opd_f64(D.ptr(totals), float(mean_tot[0]), D.ptr(totals[1]), float(mean_tot[1]),
                                     D.ptr(det2), n, D.host_f64(mean_focus), n, D.ptr(dist_err),
                                     D.ptr(dist_err2), D.ptr(sph), D.ptr(wave2), D.stream_handle()))
            res.update(dist_err2=dist_err2, sph=sph, wave2=wave2)
        else:
            _lib.check(L.akb_opd_f64(D.ptr(totals), float(mean_tot[0]), None, 0.0, None, n, None, n,
                                     D.ptr(dist_err), None, None, None, D.stream_handle()))
        return res

    # -------------------------------------------------------------- pupil for the PSF
    def pupil(self, size=128, out=None):
        """Wave2 (nm) sampled onto a size x size pupil in ray-index space (nearest ray), as OPD in
        metres plus the binary amplitude, and the pitch of the detector-2 footprint.

        This stands in for griddata(cubic) + plane correction + rotate_with_nan of the driver
        (:3689-3710, psf_calc :1121-1188; SURVEY.md §8 rows f1/f4, not yet built): the ray grid is
        a smooth deformed structured grid, so index-space sampling keeps the pupil's shape.
        Multi-GPU: each shard fills its rows and the pieces are summed over ranks."""
        n = self.n
        idx = torch.div(torch.arange(size, device=self.dev) * (n - 1), size - 1, rounding_mode="floor")
        r0, rows = self.shard.row0, self.shard.rows
        w = self.last["wave2"].view(rows, n)
        mine = (idx >= r0) & (idx < r0 + rows)
        opd = torch.zeros((size, size), dtype=D.F64, device=self.dev) if out is None else out.zero_()
        sel = idx[mine] - r0
        opd[mine] = w.index_select(0, sel).index_select(1, idx) * 1e-9
        d2 = self.last["detcenter2"]
        ext = torch.stack([torch.amax(d2[1]), -torch.amin(d2[1]), torch.amax(d2[2]), -torch.amin(d2[2])])
        ext = self.comm.allreduce_max(ext) if self.comm.world > 1 else ext
        opd = self.comm.allreduce_sums(opd) if self.comm.world > 1 else opd
        amp = torch.isfinite(opd).to(D.F64)
        e = ext.cpu().numpy()
        dx = (e[0] + e[1]) / (size - 1)
        dy = (e[2] + e[3]) / (size - 1)
        return opd, amp, dx, dy

    # -------------------------------------------------------------- accounting
    def intersections_per_run(self):
        """Ray-surface intersections computed per run by this shard: 2 passes x K mirrors."""
        return 2 * len(self.g.mirrors) * self.n_local
