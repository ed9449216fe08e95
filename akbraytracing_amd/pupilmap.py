"""Pupil-map post-processing of the 'ray_wave' driver, device-backed.

plane_correction_with_nan_and_outlier_filter (AKB_raytrace_20250312.py:9630-9693) removes the
best plane from the gridded wavefront: a quadratic least-squares fit over the finite points, the
residual's 3-sigma outliers dropped, a plane refit over the rest, the plane subtracted with the
NaNs kept. The reference fits with scipy's curve_fit (Levenberg-Marquardt on the same linear
models); the fits are linear least squares, so their solutions are the normal-equation
solutions: the device forms the sums (akb_map_moments_f64), the host solves 5 x 5 and 3 x 3
systems, the device subtracts (akb_plane_subtract_f64). Agreement with the reference is to the
fit's rounding (~1e-13 of the map's range), not bit for bit: curve_fit's iterations stop at their
own tolerance.

match_legendre_multi (legendre_fit.py:75-92) projects a square map on unit-norm Legendre
products: the rows numpy sums are formed on the device (akb_legendre_rows_f64) and summed in
numpy's pairwise order (akb_pairwise_sum_f64), so the inner products are the reference's own.
"""
import numpy as np
import torch
from scipy.special import legendre

from . import _lib
from . import device as D
from .reduce import RowSums

_SLOT = {}
for _r in range(5):
    for _c in range(_r, 5):
        _SLOT[(_r, _c)] = _r * 5 - _r * (_r - 1) // 2 + (_c - _r)


def _as_dev(m):
    if isinstance(m, torch.Tensor):
        return m.to(device=D.device(), dtype=D.F64).contiguous()
    return D.to_dev(np.ascontiguousarray(m, dtype=np.float64))


def _normal_solve(mom, nb):
    A = np.empty((nb, nb))
    for r in range(nb):
        for c in range(nb):
            A[r, c] = mom[_SLOT[(min(r, c), max(r, c))]]
    b = mom[15:15 + nb]
    return np.linalg.solve(A, b)


class _Moments:
    """akb_map_moments_f64 over k maps at once: one launch per map, one host copy for all of them."""

    def __init__(self, dev, k=1):
        L = _lib.lib()
        self.k = k
        self.work = torch.empty((k, int(L.akb_moments_work_bytes()) // 8), dtype=D.F64, device=dev)
        self.out = torch.empty((k, 21), dtype=D.F64, device=dev)

    def __call__(self, zs, nb, coefs=None, thr=None, mode=0, means=None):
        L = _lib.lib()
        for j, z in enumerate(zs):
            ny, nx = int(z.shape[0]), int(z.shape[1])
            _lib.check(L.akb_map_moments_f64(D.ptr(z), ny, nx, nb, D.ptr(coefs[j] if coefs else None),
                                             float(thr[j] if thr else 0.0), mode, float(means[j] if means else 0.0),
                                             D.ptr(self.out[j]), D.ptr(self.work[j]), D.stream_handle()))
        return self.out[:len(zs)].cpu().numpy()


def _plane_corrections(zs, sigma_threshold=3):
    """plane_correction_with_nan_and_outlier_filter of each map in zs (device tensors), in lockstep so
    each of the four stages costs one host copy for all the maps."""
    mom = _Moments(zs[0].device, len(zs))
    m0 = mom(zs, 5)
    for m in m0:
        if m[20] < 5:
            # curve_fit refuses fewer points than parameters (:9667)
            raise TypeError(f"Improper input: func (m=5) must not exceed the data count N={int(m[20])}")
    c1 = [torch.from_numpy(_normal_solve(m, 5)).to(zs[0].device) for m in m0]
    cnt = mom(zs, 5, c1, mode=1)
    means = [c[0] / c[20] for c in cnt]
    ss = mom(zs, 5, c1, mode=2, means=means)
    thr = [sigma_threshold * np.sqrt(v[0] / c[20]) for v, c in zip(ss, cnt)]
    m1 = mom(zs, 3, c1, thr=thr)
    outs = []
    for z, m in zip(zs, m1):
        if m[20] < 3:
            raise TypeError(f"Improper input: func (m=3) must not exceed the data count N={int(m[20])}")
        p2 = torch.from_numpy(_normal_solve(m, 3)).to(z.device)
        out = torch.empty_like(z)
        _lib.check(_lib.lib().akb_plane_subtract_f64(D.ptr(z), int(z.shape[0]), int(z.shape[1]), D.ptr(p2),
                                                     D.ptr(out), D.stream_handle()))
        outs.append(out)
    return outs


def plane_correction_with_nan_and_outlier_filter(data, sigma_threshold=3):
    """Drop-in for the reference function: same arguments, same result (NaNs kept). A torch
    input returns a device tensor, a numpy input a numpy array."""
    as_torch = isinstance(data, torch.Tensor)
    z = _as_dev(data)
    if z.dim() != 2:
        raise ValueError("data must be 2-D")
    out = _plane_corrections([z], sigma_threshold)[0]
    return out if as_torch else out.cpu().numpy()


def legendre_orders(order):
    """(ny, nx) pairs in match_legendre_multi's order (legendre_fit.py:82-90)."""
    return [(i - j, j) for i in range(order) for j in range(i + 1)]


def match_legendre_multi(data, order):
    """Drop-in for legendre_fit.match_legendre_multi: (fit_datas (K, n, n), inner_products (K,),
    orders [(ny, nx), ...]). numpy in, numpy out; a torch input returns device tensors."""
    as_torch = isinstance(data, torch.Tensor)
    z = _as_dev(data)
    n0, n1 = int(z.shape[0]), int(z.shape[1])
    if n0 != n1:
        # the reference's Z is (n1, n0) against data (n0, n1): numpy refuses the product
        raise ValueError(f"operands could not be broadcast together with shapes ({n1},{n0}) ({n0},{n1})")
    n, order = n0, int(order)
    orders = legendre_orders(order)
    K = len(orders)
    x = np.linspace(-1, 1, n)
    tab = np.stack([legendre(k)(x) for k in range(order)])  # scipy's poly1d values, as the reference
    dev = z.device
    pxy = torch.from_numpy(np.ascontiguousarray(tab)).to(dev)
    ordt = torch.tensor(np.array(orders, dtype=np.int32).ravel(), device=dev)
    rows = torch.empty((K, n * n), dtype=D.F64, device=dev)
    L = _lib.lib()
    sums = RowSums()

    def run(mode, s=None, c=None):
        _lib.check(L.akb_legendre_rows_f64(D.ptr(z), n, K, order, D.ptr(pxy), D.ptr(pxy), D.ptr(ordt), D.ptr(s),
                                           D.ptr(c), mode, D.ptr(rows), D.stream_handle()))

    run(0)
    s, _ = sums(rows, nan=True)
    s = s.clone()
    run(1, s)
    c, _ = sums(rows, nan=True)
    c = c.clone()
    run(2, s, c)
    fits = rows.view(K, n, n)
    if as_torch:
        return fits, c, [tuple(o) for o in orders]
    return fits.cpu().numpy(), c.cpu().numpy(), [tuple(o) for o in orders]


def wave_maps(detcenter2, dist_err2, wave2, ray_num_H, ray_num_V, grid_num_H=None, grid_num_V=None, **grid_kw):
    """The driver's gridding step (AKB_raytrace_20250312.py:3653-3696) on the device:
    grid_H, grid_V = meshgrid(linspace(min, max) of the hits' y / z), matrixDistError2 and
    matrixWave2 by cubic griddata (one triangulation for both), matrixWave2 -= nanmean, then both
    plane-corrected. detcenter2 (3, n), dist_err2 / wave2 (n,) in ray order (n = V * H).
    grid_num_H / grid_num_V: the output grid's size when it is not the ray grid's (the driver uses
    ray_num for both; bench.py grids 1e7 hits onto its 128 x 128 pupil).
    grid_kw: passed to CubicGrid (diag_override).
    Returns a dict of device tensors (the grids as numpy)."""
    from .griddata import CubicGrid
    d2 = _as_dev(detcenter2)
    y, z = d2[1].contiguous(), d2[2].contiguous()
    cg = CubicGrid(y, z, int(ray_num_V), int(ray_num_H), **grid_kw)
    ext = cg.extent  # min / max of the hits' y and z (on the lattice's boundary ring, exactly)
    gx = np.linspace(ext[0], ext[1], int(grid_num_H or ray_num_H))
    gy = np.linspace(ext[2], ext[3], int(grid_num_V or ray_num_V))
    grid_H, grid_V = np.meshgrid(gx, gy)
    vals = torch.stack([_as_dev(dist_err2).reshape(-1), _as_dev(wave2).reshape(-1)])
    maps = cg.interp(vals, gx, gy)
    m_dist, m_wave = maps[0], maps[1]
    s, c = RowSums()(m_wave.reshape(1, -1), nan=True)
    m_wave = m_wave - (s / c.to(D.F64))[0]  # np.nanmean: nansum / count
    w_c, d_c = _plane_corrections([m_wave.contiguous(), m_dist.contiguous()])
    return dict(grid_H=grid_H, grid_V=grid_V, matrixDistError2=m_dist, matrixWave2=m_wave,
                matrixWave2_Corrected=w_c, matrixDistError2_Corrected=d_c, sweeps=cg.sweeps)


def wave_pupil(detcenter2, wave2, ray_num_H, ray_num_V, grid_num_H=None, grid_num_V=None, **grid_kw):
    """The PSF's half of the driver's gridding step (AKB_raytrace_20250312.py:3653-3696): grid,
    griddata(cubic) of Wave2, minus its nanmean, plane-corrected - matrixWave2_Corrected, the map
    psf_calc transforms (:3698-3700). The same arithmetic as wave_maps' Wave2 (one value set on the
    triangulation instead of two); matrixDistError2, the driver's other map, feeds no PSF.
    detcenter2 may also be the pair (y, z) of its rows 1 and 2.
    Returns (matrixWave2_Corrected device tensor, grid_H, grid_V, gradient sweeps)."""
    from .griddata import CubicGrid
    if isinstance(detcenter2, (tuple, list)):
        y, z = (_as_dev(a).reshape(-1) for a in detcenter2)
    else:
        d2 = _as_dev(detcenter2)
        y, z = d2[1].contiguous(), d2[2].contiguous()
    cg = CubicGrid(y, z, int(ray_num_V), int(ray_num_H), **grid_kw)
    ext = cg.extent
    gx = np.linspace(ext[0], ext[1], int(grid_num_H or ray_num_H))
    gy = np.linspace(ext[2], ext[3], int(grid_num_V or ray_num_V))
    grid_H, grid_V = np.meshgrid(gx, gy)
    m_wave = cg.interp(_as_dev(wave2).reshape(1, -1), gx, gy)[0]
    s, c = RowSums()(m_wave.reshape(1, -1), nan=True)
    m_wave = m_wave - (s / c.to(D.F64))[0]
    return _plane_corrections([m_wave.contiguous()])[0], grid_H, grid_V, cg.sweeps


POST_PARAMS = 20  # akb_pupil_post_f64's parameter block (include/akb_raytrace.h)


def pupil_post(m, sigma_threshold=3, out=None, stream=None):
    """The driver's chain from a gridded Wave2 map to compute_psf_fft's input on the device, no host
    round trip (akb_pupil_post_f64: the one-workgroup post, the prefilter, the rotation): matrixWave2 - nanmean -> plane correction ->
    psf_calc's rotation estimate and rotate_with_nan (:3690-3700, :9630-9693, :1121-1188).
    m: (ny, nx) device map, ny * nx <= 65536. out: optional dict of preallocated buffers.
    Returns dict(corrected, rotated, opd, params) of device tensors; params[17] holds error flags
    (bit 0: too few points for the fits, bit 1: a singular normal system), read by the caller when
    it can wait (pupil_post_check); params[18], [19]: the input map's nanmin and nanmax."""
    L = _lib.lib()
    m = _as_dev(m)
    ny, nx = int(m.shape[0]), int(m.shape[1])
    o = out if out is not None else {}
    for k in ("corrected", "rotated", "opd"):
        if k not in o or tuple(o[k].shape) != (ny, nx):
            o[k] = torch.empty((ny, nx), dtype=D.F64, device=m.device)
    nw = int(L.akb_pupil_post_work_bytes(ny, nx)) // 8
    if "work" not in o or o["work"].numel() < nw:
        o["work"] = torch.empty(nw, dtype=D.F64, device=m.device)
    if "params" not in o:
        o["params"] = torch.empty(POST_PARAMS, dtype=D.F64, device=m.device)
    _lib.check(L.akb_pupil_post_f64(D.ptr(m), ny, nx, float(sigma_threshold), D.ptr(o["corrected"]),
                                    D.ptr(o["rotated"]), D.ptr(o["opd"]), D.ptr(o["work"]), D.ptr(o["params"]),
                                    D.stream_handle(stream)))
    return o


def pupil_post_check(params):
    """Raise as the host chain would for a pupil_post parameter block (host copy or device tensor)."""
    p = params.cpu().numpy() if isinstance(params, torch.Tensor) else np.asarray(params)
    flags = int(p[17])
    if flags & 1:
        raise TypeError(f"Improper input: the plane fit needs more finite points (N={int(p[1])})")
    if flags & 2:
        raise np.linalg.LinAlgError("Singular matrix")
