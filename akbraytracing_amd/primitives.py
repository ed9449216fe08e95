"""Drop-in GPU versions of the reference's ray primitives, with the reference's signatures.

Each function takes what the reference's takes (numpy arrays, lists of coefficients; torch
tensors are accepted too and stay on the device), runs ONE HIP kernel of libakb_hip.so, and
returns what the reference returns, including its value-level error rules:

  mirr_ray_intersection  EllipseRaytrace3D.py:18-45 / AKB_raytrace_20250312.py:444-471
                         all-NaN output when any discriminant is not > 0 (:457-459)
  norm_vector            EllipseRaytrace3D.py:61-71 / AKB_raytrace_20250312.py:626-636
  reflect_ray            EllipseRaytrace3D.py:47-55 / AKB_raytrace_20250312.py:501-509
  normalize_vector       EllipseRaytrace3D.py:57-59 / AKB_raytrace_20250312.py:530-532
                         returns its input unchanged when any norm is 0
  plane_ray_intersection EllipseRaytrace3D.py:145-157 / AKB_raytrace_20250312.py:873-885
  rotate_vectors / rotate_points  AKB_raytrace_20250312.py:917-943

Results are bit-identical to the reference's numpy evaluation (fixtures in tests/golden).
Inputs are converted to float64 (the reference's np.longdouble initial_params path, :14075, is
not reproduced: fp64 only). There is no CPU fallback: without a GPU these raise.
"""
import numpy as np
import torch

from . import _lib
from . import device as D


def _shape3(a):
    shp = tuple(a.shape)
    if len(shp) == 1:
        if shp[0] != 3:
            raise ValueError("expected 3 components")
        return None
    if len(shp) != 2 or shp[0] != 3:
        raise ValueError("expected a (3, N) array")
    return shp[1]


def _view(t):
    """(pointer, ld, inc) of a contiguous (3, N) / (3,) device tensor; one column broadcasts."""
    if t.dim() == 1:
        return D.ptr(t), 1, 0
    n = t.shape[1]
    return D.ptr(t), n, (1 if n > 1 else 0)


def _src_cols(src_cols, other_cols):
    if src_cols is None:
        raise IndexError("too many indices for array: array is 1-dimensional, but 2 were indexed")
    if other_cols is not None and other_cols not in (1, src_cols):
        raise ValueError(f"could not broadcast input array from shape ({other_cols},) into shape ({src_cols},)")
    return src_cols


def _bcast_cols(a, b):
    ca = 1 if a is None else a
    cb = 1 if b is None else b
    if ca != cb and 1 not in (ca, cb):
        raise ValueError(f"operands could not be broadcast together with shapes (3,{ca}) (3,{cb})")
    return max(ca, cb)


def _coeffs(coeffs, lo=0, hi=10):
    vals = list(coeffs)[lo:hi]
    if len(vals) != hi - lo:
        raise ValueError("expected 10 quadric coefficients")
    return D.host_f64(vals)


def _is_torch(*xs):
    return any(isinstance(x, torch.Tensor) for x in xs)


def _finish(out, shape, flags, bits, as_torch, fallback=None):
    """Apply the reference's all-or-nothing rules and return numpy (or torch) output."""
    f = int(flags.item())
    if f & bits:
        if fallback is not None:
            return fallback()
        if as_torch:
            return torch.full(shape, float("nan"), dtype=D.F64, device=out.device)
        return np.full(shape, np.nan)
    out = out.reshape(shape)
    return out if as_torch else out.cpu().numpy()


def mirr_ray_intersection(coeffs, ray, source, negative=False):
    L = _lib.lib()
    as_torch = _is_torch(ray, source)
    d, s = D.to_dev(ray), D.to_dev(source)
    n = _src_cols(_shape3(s), _shape3(d))
    out = D.empty((3, n))
    fl = D.flags_tensor()
    dp, dld, dinc = _view(d)
    sp, sld, sinc = _view(s)
    _lib.check(L.akb_isect_f64(_coeffs(coeffs), dp, dld, dinc, sp, sld, sinc, int(bool(negative)), n,
                               D.ptr(out), n, D.ptr(fl), D.stream_handle()))
    return _finish(out, tuple(s.shape), fl, _lib.FLAG_MISS, as_torch)


def norm_vector(coeffs, point):
    L = _lib.lib()
    as_torch = _is_torch(point)
    p = D.to_dev(point)
    pc = _shape3(p)
    n = 1 if pc is None else pc
    out = D.empty((3, n))
    fl = D.flags_tensor()
    pp, pld, pinc = _view(p)
    c = _coeffs(coeffs)
    _lib.check(L.akb_normal_f64(c, pp, pld, pinc, n, D.ptr(out), n, 1, D.ptr(fl), D.stream_handle()))

    def raw():  # any zero-norm gradient: the reference returns the unnormalised gradient
        _lib.check(L.akb_normal_f64(c, pp, pld, pinc, n, D.ptr(out), n, 0, D.ptr(fl), D.stream_handle()))
        o = out.reshape(tuple(p.shape))
        return o if as_torch else o.cpu().numpy()
    return _finish(out, tuple(p.shape), fl, _lib.FLAG_ZERO_NORMAL, as_torch, fallback=raw)


def reflect_ray(ray, N):
    L = _lib.lib()
    as_torch = _is_torch(ray, N)
    d, v = D.to_dev(ray), D.to_dev(N)
    n = _bcast_cols(_shape3(d), _shape3(v))
    shape = tuple(torch.broadcast_shapes(tuple(d.shape), tuple(v.shape)))
    out = D.empty((3, n))
    fl = D.flags_tensor()
    dp, dld, dinc = _view(d)
    vp, vld, vinc = _view(v)
    _lib.check(L.akb_reflect_f64(dp, dld, dinc, vp, vld, vinc, n, D.ptr(out), n, 1, D.ptr(fl),
                                 D.stream_handle()))

    def raw():
        _lib.check(L.akb_reflect_f64(dp, dld, dinc, vp, vld, vinc, n, D.ptr(out), n, 0, D.ptr(fl),
                                     D.stream_handle()))
        o = out.reshape(shape)
        return o if as_torch else o.cpu().numpy()
    return _finish(out, shape, fl, _lib.FLAG_ZERO_REFLECT, as_torch, fallback=raw)


def normalize_vector(vector):
    L = _lib.lib()
    as_torch = _is_torch(vector)
    v = D.to_dev(vector)
    vc = _shape3(v)
    n = 1 if vc is None else vc
    out = D.empty((3, n))
    fl = D.flags_tensor()
    vp, vld, vinc = _view(v)
    _lib.check(L.akb_normalize_f64(vp, vld, vinc, n, D.ptr(out), n, D.ptr(fl), D.stream_handle()))
    return _finish(out, tuple(v.shape), fl, _lib.FLAG_ZERO_DIR, as_torch, fallback=lambda: vector)


def plane_ray_intersection(coeffs, ray, source):
    L = _lib.lib()
    as_torch = _is_torch(ray, source)
    d, s = D.to_dev(ray), D.to_dev(source)
    n = _src_cols(_shape3(s), _shape3(d))
    out = D.empty((3, n))
    dp, dld, dinc = _view(d)
    sp, sld, sinc = _view(s)
    _lib.check(L.akb_plane_isect_f64(_coeffs(coeffs, 6, 10), dp, dld, dinc, sp, sld, sinc, n, D.ptr(out), n,
                                     D.stream_handle()))
    out = out.reshape(tuple(s.shape))
    return out if as_torch else out.cpu().numpy()


def segment_length(a, b):
    """np.linalg.norm(b - a, axis=0) (the OPL segments, AKB_raytrace_20250312.py:2884-2897)."""
    L = _lib.lib()
    as_torch = _is_torch(a, b)
    x, y = D.to_dev(a), D.to_dev(b)
    n = _bcast_cols(_shape3(x), _shape3(y))
    out = D.empty((n,))
    xp, xld, xinc = _view(x)
    yp, yld, yinc = _view(y)
    _lib.check(L.akb_seglen_f64(xp, xld, xinc, yp, yld, yinc, n, D.ptr(out), D.stream_handle()))
    return out if as_torch else out.cpu().numpy()


def rotation_matrices(theta_y, theta_z):
    """R_y and R_z of rotate_vectors (AKB_raytrace_20250312.py:917-927), formed with numpy on the
    host exactly as the reference forms them."""
    cy, sy = np.cos(theta_y), np.sin(theta_y)
    cz, sz = np.cos(theta_z), np.sin(theta_z)
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]], dtype=np.float64)
    rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]], dtype=np.float64)
    return ry, rz


def _rotate(v_in, center, theta_y, theta_z):
    L = _lib.lib()
    as_torch = _is_torch(v_in)
    v = D.to_dev(v_in)
    vc = _shape3(v)
    n = 1 if vc is None else vc
    ry, rz = rotation_matrices(theta_y, theta_z)
    out = D.empty((3, n))
    vp, vld, vinc = _view(v)
    c = None if center is None else D.host_f64(np.asarray(center, dtype=np.float64).ravel()[:3])
    _lib.check(L.akb_rotate_f64(D.host_f64(ry.ravel()), D.host_f64(rz.ravel()), c, vp, vld, vinc, n, D.ptr(out),
                                n, D.stream_handle()))
    out = out.reshape(tuple(v.shape))
    return out if as_torch else out.cpu().numpy()


def rotate_vectors(vector, theta_y, theta_z):
    return _rotate(vector, None, theta_y, theta_z)


def rotate_points(points, focus_apprx, theta_y, theta_z):
    return _rotate(points, focus_apprx, theta_y, theta_z)
