"""Device-resident mirror-chain tracing (the fused HIP path behind the drivers' two passes).

A ray grid is never materialised: the chain kernel generates each ray's direction from two
1-D tables, normalize(1, tan_h[ih], tan_v[iv]) at flat index iv*n_h + ih, exactly as the
drivers build phai0 (AKB_raytrace_20250312.py:2711-2717; KB_debug :10964-10970), then runs
intersect -> normal -> reflect through K quadrics with all intermediate state in registers,
accumulates the optical path ((d01 + d12) + d23) + ... left to right (:2884-2897, :3625), and
writes only what the caller asks for.

The reference's value rules are kept exactly: the kernel raises per-mirror flags for any
non-positive discriminant or zero norm, and a flagged pass is re-run stage by stage through
the drop-in primitives, which apply the all-NaN / passthrough rules of :457 and :530-532.
"""
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from . import device as D
from . import primitives as P


@dataclass
class Mirror:
    """A quadric a x^2 + b y^2 + c z^2 + d xy + e xz + f yz + g x + h y + i z + j = 0."""
    coeffs: list
    negative: bool = False

    def __post_init__(self):
        self.coeffs = [float(c) for c in self.coeffs]
        if len(self.coeffs) != 10:
            raise ValueError("a mirror needs 10 quadric coefficients")


@dataclass
class ChainOutputs:
    """Device tensors written by one chain launch (None when not requested)."""
    flags: torch.Tensor
    hits: torch.Tensor = None        # (K, 3, n)
    last_hit: torch.Tensor = None    # (3, n)
    dir_out: torch.Tensor = None     # (3, n)
    det: torch.Tensor = None         # (3, n)
    opl: torch.Tensor = None         # (n,)  sum of the K segment lengths
    atan: torch.Tensor = None        # (2, n) arctan(Ry/Rx), arctan(Rz/Rx)
    samp_h: torch.Tensor = None      # slope samples of the middle row
    samp_v: torch.Tensor = None      # slope samples of the middle column
    extra: dict = field(default_factory=dict)


def _fill_desc(desc, mirrors, det_ghij):
    if not 0 < len(mirrors) <= _lib.MAX_MIRRORS:
        raise ValueError(f"1..{_lib.MAX_MIRRORS} mirrors supported")
    desc.n_mirrors = len(mirrors)
    for k, m in enumerate(mirrors):
        desc.negative[k] = int(bool(m.negative))
        for j in range(10):
            desc.coeffs[k][j] = m.coeffs[j]
    if det_ghij is not None:
        for j in range(4):
            desc.det_ghij[j] = float(det_ghij[j])


class ChainLaunch:
    """A prepared fused-chain launch: the descriptor and its device buffers are built once and
    the launch can be repeated (the tables / source / sink contents may change between launches,
    their addresses may not). trace_chain() is the one-shot form."""

    def __init__(self, mirrors, *, tan_h=None, tan_v=None, row0=0, n_rays=None, dirs=None, src=(0.0, 0.0, 0.0),
                 det_ghij=None, want=("last_hit", "dir_out"), samples=None, out=None, sink=None, flags=None,
                 samples_buf=None, pert=None, ray0=None):
        dev = D.device()
        desc = _lib.ChainDesc()
        _fill_desc(desc, mirrors, det_ghij)
        self.keep = [tan_h, tan_v, dirs, sink]
        if dirs is None:
            n_h, n_v = tan_h.shape[0], tan_v.shape[0]
            ray0 = row0 * n_h if ray0 is None else int(ray0)
            n = n_h * n_v - ray0 if n_rays is None else n_rays
            desc.dir = None
            desc.tan_h, desc.tan_v = D.ptr(tan_h), D.ptr(tan_v)
            desc.n_h, desc.n_v, desc.ray0 = n_h, n_v, ray0
        else:
            n = dirs.shape[1]
            desc.dir, desc.dir_ld, desc.dir_inc = D.ptr(dirs), n, 1
            desc.n_h, desc.n_v = 1, n
        desc.n_rays = n
        if isinstance(src, torch.Tensor) and src.dim() == 2:
            desc.org, desc.org_ld, desc.org_inc = D.ptr(src), src.shape[1], 1
            self.keep.append(src)
        else:
            desc.org = None
            s = [float(x) for x in np.asarray(src, dtype=np.float64).ravel()[:3]]
            for j in range(3):
                desc.src[j] = s[j]
        out = dict(out or {})
        K = len(mirrors)

        def buf(name, shape):
            t = out.get(name)
            if t is None or tuple(t.shape) != tuple(shape):
                t = torch.empty(shape, dtype=D.F64, device=dev)
            out[name] = t
            return t

        if flags is None:
            flags = torch.zeros(1, dtype=torch.int32, device=dev)
        res = ChainOutputs(flags=flags)
        if "hits" in want:
            res.hits = buf("hits", (K, 3, n))
            desc.hits, desc.hits_ld = D.ptr(res.hits), n
        if "last_hit" in want:
            res.last_hit = buf("last_hit", (3, n))
            desc.last_hit, desc.last_hit_ld = D.ptr(res.last_hit), n
        if "dir_out" in want:
            res.dir_out = buf("dir_out", (3, n))
            desc.dir_out, desc.dir_out_ld = D.ptr(res.dir_out), n
        if "det" in want:
            if det_ghij is None:
                raise ValueError("det requested without a detector plane")
            res.det = buf("det", (3, n))
            desc.det_out, desc.det_out_ld = D.ptr(res.det), n
        if "opl" in want:
            res.opl = buf("opl", (n,))
            desc.opl = D.ptr(res.opl)
        if "atan" in want:
            res.atan = buf("atan", (2, n))
            desc.atan_h = D.ptr(res.atan)
            desc.atan_v = D.ptr(res.atan[1])
        desc.samp_h_begin = desc.samp_h_end = 0
        desc.samp_v_col = -1
        if samples is not None:
            hb, he, vc = samples
            nh = max(he - hb, 0)
            nv = tan_v.shape[0] if vc is not None else 0
            # one buffer so the host reads both pick lists with one copy
            if samples_buf is not None:
                if samples_buf.numel() != nh + nv or samples_buf.dtype != D.F64:
                    raise ValueError("samples_buf must hold the middle-row range plus one column (float64)")
                samples_buf.fill_(float("nan"))
                res.extra["samples"] = samples_buf
            else:
                res.extra["samples"] = torch.full((nh + nv,), float("nan"), dtype=D.F64, device=dev)
            res.samp_h = res.extra["samples"][:nh]
            desc.samp_h, desc.samp_h_begin, desc.samp_h_end = D.ptr(res.samp_h), hb, he
            if vc is not None:
                res.samp_v = res.extra["samples"][nh:]
                desc.samp_v, desc.samp_v_col = D.ptr(res.samp_v), vc
        desc.flags = D.ptr(res.flags)
        if sink is not None:
            if det_ghij is None:
                raise ValueError("the chain sink reduces detector hits: give det_ghij")
            desc.sink = sink.desc
        if pert is not None:
            if dirs is not None or "opl" not in want:
                raise ValueError("the OPL perturbation applies to grid rays with want containing 'opl'")
            ph, pv = pert
            if ph.shape[0] != pv.shape[0] or ph.shape[1] != desc.n_h or pv.shape[1] != desc.n_v:
                raise ValueError("perturbation tables must be (terms, n_h) and (terms, n_v)")
            desc.pert_h, desc.pert_v, desc.pert_terms = D.ptr(ph), D.ptr(pv), int(ph.shape[0])
            self.keep += [ph, pv]
        res.extra["buffers"] = out
        self.desc, self.res = desc, res

    def launch(self, stream=None, reset_flags=True):
        if reset_flags:
            self.res.flags.zero_()
        _lib.check(_lib.lib().akb_trace_chain_f64(self.desc, D.stream_handle(stream)))
        return self.res


def trace_chain(mirrors, *, stream=None, **kw):
    """Run one fused chain launch.

    Rays: either the grid (tan_h, tan_v device tensors; flat rays ray0 .. + n_rays, ray0 defaulting
    to row0 * n_h) or explicit
    `dirs` (3, n) device tensor. Source: a 3-vector (constant) or a (3, n) device tensor.
    want: subset of {"hits", "last_hit", "dir_out", "det", "opl", "atan"}.
    samples: (h_begin, h_end, v_col) flat-index range / column whose exit slopes to record.
    flags / samples_buf: optional caller-owned int32 flag word and float64 pick buffer (RayWave
        places the flag words right after the picks so one copy brings both to the host).
    pert: optional (pert_h, pert_v) device tables of a legendre.LegendrePerturbation, added to
        each grid ray's OPL (BASELINE config 5).
    out: optional dict of preallocated tensors keyed like ChainOutputs fields (reused buffers).
    sink: optional reduce.LeafSink(5, n_rays, nan_mask=0b00011) fed with (arctan(Ry/Rx),
        arctan(Rz/Rx), det_x, det_y, det_z) — the tilt means without writing those rows.
    """
    return ChainLaunch(mirrors, **kw).launch(stream=stream, reset_flags=False)


def staged_chain(mirrors, dirs, src, with_segments=False):
    """The chain as the reference runs it, one primitive per stage (exact value rules).
    Used when the fused kernel flags a miss or a zero norm. dirs, src: (3, n) device tensors."""
    hits, segs = [], []
    ray, org = dirs, src
    for m in mirrors:
        p = P.mirr_ray_intersection(m.coeffs, ray, org, negative=m.negative)
        if with_segments:
            segs.append(P.segment_length(org, p))
        ray = P.reflect_ray(ray, P.norm_vector(m.coeffs, p))
        org = p
        hits.append(p)
    return hits, ray, segs


def grid_dirs(tan_h, tan_v):
    """phai0 on the device (3, n_h*n_v), normalised exactly as the reference normalises it."""
    n_h, n_v = tan_h.shape[0], tan_v.shape[0]
    phai0 = torch.empty((3, n_h * n_v), dtype=D.F64, device=tan_h.device)
    phai0[0] = 1.0
    phai0[1] = tan_h.repeat(n_v)
    phai0[2] = tan_v.repeat_interleave(n_h)
    return P.normalize_vector(phai0)
