"""CPU oracle for the AKB hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
It is the checker the HIP path is compared against, never the thing measured or shipped: the
product package (akbraytracing_amd) does not import it and has no CPU fallback.

Contents
  * the reference's numpy primitives restated in C (akb_oracle.c, gcc -O2 -ffp-contract=off,
    OpenMP) with the reference's Python signatures and its all-or-nothing NaN / passthrough
    rules (EllipseRaytrace3D.py:18-71, :145-157; AKB_raytrace_20250312.py:444-532, :873-943);
  * numpy's float64 sum (oracle_np_sum) restated, used to pin the GPU reduction;
  * pipeline.py — the hot-path slice of plot_result_debug / KB_debug (ray grid, two passes,
    tilt, OPD) over those primitives;
  * psf.py, huygens.py, legendre.py — numpy restatements of psf_fft.compute_psf_fft,
    Wavecalc compute_u_parallel and the legendre_fit basis.

Pinned against vectors recorded from the reference itself (tests/golden/make_golden.py);
tests/test_oracle_golden.py checks every fixture.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libakb_oracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_i64 = ctypes.c_int64


def build():
    """Compile the C restatement (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        v3 = [ctypes.c_void_p, _i64, _i64]
        L.oracle_isect.argtypes = [ctypes.c_void_p] + v3 + v3 + [ctypes.c_int, _i64, ctypes.c_void_p, _i64]
        L.oracle_isect.restype = ctypes.c_int
        L.oracle_normal.argtypes = [ctypes.c_void_p] + v3 + [_i64, ctypes.c_void_p, _i64]
        L.oracle_normal.restype = ctypes.c_int
        L.oracle_reflect.argtypes = v3 + v3 + [_i64, ctypes.c_void_p, _i64]
        L.oracle_reflect.restype = ctypes.c_int
        L.oracle_normalize.argtypes = v3 + [_i64, ctypes.c_void_p, _i64]
        L.oracle_normalize.restype = ctypes.c_int
        L.oracle_plane.argtypes = [ctypes.c_void_p] + v3 + v3 + [_i64, ctypes.c_void_p, _i64]
        L.oracle_plane.restype = None
        L.oracle_seglen.argtypes = v3 + v3 + [_i64, ctypes.c_void_p]
        L.oracle_seglen.restype = None
        L.oracle_rotate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + v3 + [
            _i64, ctypes.c_void_p, _i64]
        L.oracle_rotate.restype = None
        L.oracle_np_sum.argtypes = [ctypes.c_void_p, _i64, ctypes.c_int, ctypes.POINTER(_i64)]
        L.oracle_np_sum.restype = ctypes.c_double
        L.oracle_huygens.argtypes = [ctypes.c_void_p] * 3 + [_i64] + [ctypes.c_void_p] * 4 + [
            _i64, ctypes.c_double, ctypes.c_void_p]
        L.oracle_huygens.restype = None
        L.oracle_max_threads.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_calc_ds.argtypes = [ctypes.c_void_p, _i64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_calc_ds.restype = None
        _lib = L
    return _lib


def set_threads(n):
    lib().oracle_set_threads(int(n))


def max_threads():
    return int(lib().oracle_max_threads())


# --------------------------------------------------------------------------------------------
# argument plumbing: a (3, N) or (3,) float64 array -> (pointer, ld, inc) and its column count
# --------------------------------------------------------------------------------------------

def _as3(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if a.ndim == 1:
        if a.shape[0] != 3:
            raise ValueError("expected 3 rows")
        return a, 1, 0, None  # (array, ld, inc, ncols) broadcast column
    if a.ndim != 2 or a.shape[0] != 3:
        raise ValueError("expected a (3, N) array")
    return a, a.shape[1], (1 if a.shape[1] > 1 else 0), a.shape[1]


def _coeffs(c):
    c = np.asarray([float(x) for x in c], dtype=np.float64)
    if c.shape[0] != 10:
        raise ValueError("expected 10 quadric coefficients")
    return c


def _out_cols(src_cols, other_cols):
    # the reference writes point[0, :] = t*l + p into zeros_like(source)
    if src_cols is None:
        raise IndexError("too many indices for array: array is 1-dimensional, but 2 were indexed")
    if other_cols is not None and other_cols not in (1, src_cols):
        raise ValueError(f"could not broadcast input array from shape ({other_cols},) into shape ({src_cols},)")
    return src_cols


def _bcast_cols(a_cols, b_cols):
    ca = 1 if a_cols is None else a_cols
    cb = 1 if b_cols is None else b_cols
    if ca != cb and 1 not in (ca, cb):
        raise ValueError(f"operands could not be broadcast together ({ca},) ({cb},)")
    return max(ca, cb)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------------------------
# the reference primitives (same signatures and value semantics)
# --------------------------------------------------------------------------------------------

def mirr_ray_intersection(coeffs, ray, source, negative=False):
    c = _coeffs(coeffs)
    d, dld, dinc, dn = _as3(ray)
    s, sld, sinc, sn = _as3(source)
    n = _out_cols(sn, dn)
    shape = np.asarray(source).shape
    out = np.empty((3, n))
    lib().oracle_isect(_ptr(c), _ptr(d), dld, dinc, _ptr(s), sld, sinc, int(bool(negative)), n, _ptr(out), n)
    return out.reshape(shape)


def norm_vector(coeffs, point):
    c = _coeffs(coeffs)
    p, pld, pinc, pn = _as3(point)
    n = pn if pn is not None else 1
    out = np.empty((3, n))
    lib().oracle_normal(_ptr(c), _ptr(p), pld, pinc, n, _ptr(out), n)
    return out.reshape(np.asarray(point).shape)


def reflect_ray(ray, N):
    d, dld, dinc, dn = _as3(ray)
    v, vld, vinc, vn = _as3(N)
    n = _bcast_cols(dn, vn)
    out = np.empty((3, n))
    lib().oracle_reflect(_ptr(d), dld, dinc, _ptr(v), vld, vinc, n, _ptr(out), n)
    shape = np.broadcast_shapes(np.asarray(ray).shape, np.asarray(N).shape)
    return out.reshape(shape)


def normalize_vector(vector):
    v, vld, vinc, vn = _as3(vector)
    n = vn if vn is not None else 1
    out = np.empty((3, n))
    zero = lib().oracle_normalize(_ptr(v), vld, vinc, n, _ptr(out), n)
    if zero:
        return vector
    return out.reshape(np.asarray(vector).shape)


def plane_ray_intersection(coeffs, ray, source):
    ghij = np.asarray([float(x) for x in list(coeffs)[6:10]], dtype=np.float64)
    d, dld, dinc, dn = _as3(ray)
    s, sld, sinc, sn = _as3(source)
    n = _out_cols(sn, dn)
    out = np.empty((3, n))
    lib().oracle_plane(_ptr(ghij), _ptr(d), dld, dinc, _ptr(s), sld, sinc, n, _ptr(out), n)
    return out.reshape(np.asarray(source).shape)


def seglen(a, b):
    """np.linalg.norm(b - a, axis=0)"""
    x, xld, xinc, xn = _as3(a)
    y, yld, yinc, yn = _as3(b)
    n = _bcast_cols(xn, yn)
    out = np.empty(n)
    lib().oracle_seglen(_ptr(x), xld, xinc, _ptr(y), yld, yinc, n, _ptr(out))
    return out


def rotation_matrices(theta_y, theta_z):
    """The R_y, R_z of rotate_vectors (AKB_raytrace_20250312.py:917-927), built with numpy."""
    ry = np.array([[np.cos(theta_y), 0, np.sin(theta_y)], [0, 1, 0], [-np.sin(theta_y), 0, np.cos(theta_y)]])
    rz = np.array([[np.cos(theta_z), -np.sin(theta_z), 0], [np.sin(theta_z), np.cos(theta_z), 0], [0, 0, 1]])
    return ry, rz


def rotate_vectors(vector, theta_y, theta_z):
    ry, rz = rotation_matrices(theta_y, theta_z)
    v, vld, vinc, vn = _as3(vector)
    n = vn if vn is not None else 1
    out = np.empty((3, n))
    lib().oracle_rotate(_ptr(np.ascontiguousarray(ry)), _ptr(np.ascontiguousarray(rz)), None, _ptr(v), vld,
                        vinc, n, _ptr(out), n)
    return out.reshape(np.asarray(vector).shape)


def rotate_points(points, focus_apprx, theta_y, theta_z):
    ry, rz = rotation_matrices(theta_y, theta_z)
    v, vld, vinc, vn = _as3(points)
    n = vn if vn is not None else 1
    c = np.ascontiguousarray(np.asarray(focus_apprx, dtype=np.float64))
    out = np.empty((3, n))
    lib().oracle_rotate(_ptr(np.ascontiguousarray(ry)), _ptr(np.ascontiguousarray(rz)), _ptr(c), _ptr(v), vld,
                        vinc, n, _ptr(out), n)
    return out.reshape(np.asarray(points).shape)


def np_sum(x, nan=False):
    """numpy's float64 sum of a 1-D array (np.nansum semantics with nan=True) and the count."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64).ravel())
    cnt = _i64(0)
    s = lib().oracle_np_sum(_ptr(x), x.shape[0], int(bool(nan)), ctypes.byref(cnt))
    return float(s), int(cnt.value)


def huygens_c(tx, ty, tz, sx, sy, sz, u_times_ds, k):
    """compute_u_parallel (Wavecalc_raytrace_fromData_CPU0402.py:71-85), OpenMP over targets;
    u_times_ds is the already-scaled source field (:102). Speed baseline; tolerance-checked."""
    arrs = [np.ascontiguousarray(np.asarray(a, dtype=np.float64)) for a in (tx, ty, tz, sx, sy, sz)]
    u = np.ascontiguousarray(np.asarray(u_times_ds, dtype=np.complex128))
    n, m = arrs[0].shape[0], arrs[3].shape[0]
    out = np.empty(n, dtype=np.complex128)
    lib().oracle_huygens(_ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]), n, _ptr(arrs[3]), _ptr(arrs[4]),
                         _ptr(arrs[5]), _ptr(u), m, float(k), _ptr(out))
    return out


def calc_dS(points, V, H):
    """calc_dS (AKB_raytrace_20250312.py:13418-13473) -> (V, H)."""
    p = np.ascontiguousarray(points, dtype=np.float64)
    out = np.empty((V, H))
    lib().oracle_calc_ds(_ptr(p), p.shape[1], int(V), int(H), _ptr(out))
    return out
