"""griddata(method='cubic') of the 'ray_wave' driver on the device.

The driver interpolates the per-ray DistError2 and Wave2 from the detector hits onto a regular
grid (AKB_raytrace_20250312.py:3673, :3689):

    griddata((detcenter2[1, :], detcenter2[2, :]), Wave2, (grid_H, grid_V), method='cubic')

scipy answers with a Clough-Tocher interpolant on the points' Delaunay triangulation. The points
are the ray grid's hits, a smoothly deformed n_v x n_h lattice, so CubicGrid builds that
triangulation structurally (akb_griddata.hip: cell diagonals by the in-circle test, the hull
pockets on the host, local-Delaunay checks that refuse a grid where this would not be qhull's
answer), estimates the vertex gradients by Jacobi sweeps of scipy's own local solve with
Chebyshev semi-iteration (a register-resident strip kernel, two sweeps per launch) until they stop
changing, and evaluates the patches on the device. Agreement with scipy is to rounding on the
reference's 65 x 65 run (tests/test_gpu_parity.py) and within 1e-6 of the range at 1001^2 /
3163^2 (tests/test_fullsize_gpu.py), not bit for bit: qhull's near-cocircular picks and scipy's
Gauss-Seidel iterates are not reproduced - both iterations converge to the same fixed point and
both stop at a largest relative change of 1e-6 (GRADIENT_TOL).
"""
import numpy as np
import torch

from . import _lib
from . import device as D

_F_NONCONVEX, _F_NOT_DELAUNAY, _F_POCKET, _F_POS, _F_NEG, _F_NONFINITE = 1, 2, 4, 8, 16, 32

# Stopping tolerance of the gradient iteration: the largest relative change of a Jacobi step
# (scipy's measure) below scipy's own tolerance, 1e-6. Its iterates and ours differ, so neither
# point is the other's: what parity needs is the interpolated values near the common fixed point,
# and stopping where scipy stops keeps that distance at scipy's own on every lattice (coarse grids
# included; tests/test_gpu_parity.py::test_griddata_default_tol_margin).
GRADIENT_TOL = 1e-6

# Fixed sweep count of the cone solve (interp_cone): the Chebyshev iteration contracts by ~0.27 a
# sweep, so after 12 sweeps from zero the interior gradients sit within ~2e-7 of their scale of the
# fixed point and the interpolated values within 1.7e-7 of the map's range (1001^2 C3 hits onto the
# 128^2 pupil; 1.2e-8 after 14 sweeps, for 1.3x the patch work): the PSF of that map differs from
# the converged chain's by ~1e-10 of its peak, four orders inside the north star's 1e-6
# (tests/test_gpu_parity.py::test_gradient_cone_on_the_c3_hits, tests/test_faithful_gpu.py,
# DESIGN.md §7.1). 14 is the patch kernel's largest (its (2K + 4)^2 box fills 32^2 in LDS).
CONE_SWEEPS = 12


# The cone solve's guard (FaithfulPupil, Ticket.check): its value-error estimate (akb_gd_cone_eval_f64's
# d_change[1]: the interior target cells' corner bound from the patches, and the band and pocket
# targets' value change of one more band sweep, from k_gd_eval) must stay within this fraction of
# the gridded map's range - the parity bar of the gridding against scipy (tests/test_fullsize_gpu.py).
CONE_GUARD = 1e-6


class ConeNotConverged(_lib.AKBError):
    """The fixed-K cone solve's error estimate exceeds CONE_GUARD of the map's range."""


def chebyshev_weights(count, rho=0.5):
    """omegas[k]: the weight of the sweep that reads x_k (omegas[0] unused: a plain first sweep),
    Chebyshev semi-iteration for a Jacobi spectrum in [-rho, rho]."""
    rho2 = rho * rho
    om = [1.0]
    for k in range(1, count + 1):
        om.append(2.0 / (2.0 - rho2) if k == 1 else 1.0 / (1.0 - rho2 * om[-1] / 4.0))
    return om


def _dev(a, dev, dtype=D.F64):
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dtype)


class CubicGrid:
    """The triangulation of an n_v x n_h grid of points (x, y: (n_v * n_h,) row-major), reused for
    any number of value sets and target grids."""

    def __init__(self, x, y, n_v, n_h, delaunay_tol=1e-10, diag_override=None):
        """diag_override: (cells, splits) - flat cell indices iv * (n_h - 1) + ih and the split each
        takes (0: p00-p11, 1: p01-p10) in place of the exact in-circle one, e.g. qhull's own picks in
        near-cocircular cells (tests/golden/akb_qhull_full.npz); the triangulation then is that one,
        and the sweeps, claims and patches follow it. The override is trusted: the local-Delaunay
        checks ran on the in-circle splits before it is applied and are not repeated for the cells
        it changes - it exists for the qhull golden parity tests, not for user input."""
        L = _lib.lib()
        self.dev = D.device()
        self.nv, self.nh = int(n_v), int(n_h)
        n = self.nv * self.nh
        self.x = _dev(x, self.dev).reshape(-1)
        self.y = _dev(y, self.dev).reshape(-1)
        if self.x.numel() != n or self.y.numel() != n:
            raise ValueError(f"{self.x.numel()} points do not form a {self.nv} x {self.nh} grid")
        if self.nv < 2 or self.nh < 2:
            raise ValueError("griddata needs a grid of at least 2 x 2 points")
        s = D.stream_handle()
        self.diag = torch.empty((self.nv - 1) * (self.nh - 1), dtype=torch.uint8, device=self.dev)
        self.L = 2 * (self.nh - 1) + 2 * (self.nv - 1)
        # ring x, ring y and the cell flags (int32 after them) come back to the host in one copy
        ringbuf = torch.zeros(2 * self.L + 1, dtype=D.F64, device=self.dev)
        flags = ringbuf.view(torch.int32)[4 * self.L:4 * self.L + 1]
        _lib.check(L.akb_gd_cells_f64(D.ptr(self.x), D.ptr(self.y), self.nv, self.nh, D.ptr(self.diag),
                                      float(delaunay_tol), D.ptr(flags), D.ptr(ringbuf[:self.L]),
                                      D.ptr(ringbuf[self.L:2 * self.L]), s))
        if diag_override is not None:
            cells, splits = (np.asarray(a).reshape(-1) for a in diag_override)
            if cells.size:
                if cells.min() < 0 or cells.max() >= self.diag.numel() or not np.isin(splits, (0, 1)).all():
                    raise ValueError("diag_override: cell index out of range or a split other than 0 / 1")
                self.diag[torch.from_numpy(cells.astype(np.int64)).to(self.dev)] = \
                    torch.from_numpy(splits.astype(np.uint8)).to(self.dev)
        rb = ringbuf.cpu().numpy()
        f = int(rb[2 * self.L:].view(np.int32)[0])
        if f & _F_NONFINITE:
            raise ValueError("griddata: non-finite point coordinates (a ray that missed)")
        if f & _F_NONCONVEX or (f & _F_POS and f & _F_NEG):
            raise _lib.AKBError("griddata: the points do not form a convex, unfolded lattice")
        if f & _F_NOT_DELAUNAY:
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
        rx, ry = rb[:self.L], rb[self.L:2 * self.L]
        # the point set's extent: an unfolded lattice's extremes lie on its boundary ring
        self.extent = (float(rx.min()), float(rx.max()), float(ry.min()), float(ry.max()))
        cap = self.L
        # tri (3 cap) | nbr (3 cap) | edge (L) | xptr (L + 1) | xidx (6 cap) | npk: one host buffer, one copy
        o_tri, o_nbr, o_edge, o_xptr = 0, 3 * cap, 6 * cap, 6 * cap + self.L
        o_xidx = o_xptr + self.L + 1
        o_npk = o_xidx + 6 * cap
        buf = np.zeros(o_npk + 1, np.int32)
        hp = lambda o: buf[o:].ctypes.data_as(_lib.c_vp)  # noqa: E731
        _lib.check(L.akb_gd_pockets(rx.ctypes.data_as(_lib.c_vp), ry.ctypes.data_as(_lib.c_vp), self.nv, self.nh,
                                    cap, hp(o_npk), hp(o_tri), hp(o_nbr), hp(o_edge), hp(o_xptr), hp(o_xidx)))
        self.npock = int(buf[o_npk])
        dbuf = torch.from_numpy(buf).to(self.dev)
        k = max(self.npock, 1)
        self.ptri = dbuf[o_tri:o_tri + 3 * k]
        self.pnbr = dbuf[o_nbr:o_nbr + 3 * k]
        self.edge_tri = dbuf[o_edge:o_edge + self.L]
        self.xptr = dbuf[o_xptr:o_xptr + self.L + 1]
        self.xidx = dbuf[o_xidx:o_xidx + 6 * cap]
        # the pockets' local-Delaunay check lands in a status word read with the first sweep batch
        self._status = torch.zeros(1, dtype=torch.int64, device=self.dev)
        _lib.check(L.akb_gd_check_pockets(D.ptr(self.x), D.ptr(self.y), self.nv, self.nh, D.ptr(self.diag),
                                          self.npock, D.ptr(self.ptri), D.ptr(self.pnbr), D.ptr(self.edge_tri),
                                          float(delaunay_tol), D.ptr(self._status), s))
        self._checked = False
        self._bad = False
        self.sweeps = 0

    def _check_status(self, word=None):
        """Raise if the pocket check flagged the triangulation (word: its value, already on the host)."""
        if self._checked:
            if self._bad:  # a flagged triangulation stays refused on every later call
                raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
            return
        f = int(self._status.item()) if word is None else int(word)
        self._checked = True
        self._bad = bool(f & (_F_NOT_DELAUNAY | _F_POCKET))
        if self._bad:
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")

    def _tri_args(self):
        return (D.ptr(self.x), D.ptr(self.y), self.nv, self.nh, D.ptr(self.diag), self.npock, D.ptr(self.ptri),
                D.ptr(self.pnbr), D.ptr(self.edge_tri))

    def gradients(self, values, tol=GRADIENT_TOL, maxiter=400, check_every=8, adaptive=True):
        """estimate_gradients_2d_global for (nvals, n) values: (nvals, n, 2) device tensor. Jacobi
        sweeps of scipy's local solve with Chebyshev semi-iteration for a spectrum in [-1/2, 1/2] (the
        local problem is block diagonally dominant by a factor 2), ~0.27 error contraction per sweep,
        two sweeps per launch of the register kernel (k_gd_sweeps). The sweeps stop after the first
        batch holding one whose largest relative change (scipy's measure of a Jacobi step) is below
        tol (GRADIENT_TOL); with adaptive, batches after the first are sized from the observed decay
        rate."""
        L = _lib.lib()
        if self._checked:
            self._check_status()  # re-raises for a triangulation the pocket check flagged
        f = _dev(values, self.dev)
        f = f.reshape(-1, self.nv * self.nh).contiguous()
        nvals = int(f.shape[0])
        shape = (nvals, self.nv * self.nh, 2)
        change = torch.zeros(maxiter + 1, dtype=torch.int64, device=self.dev)
        s = D.stream_handle()
        omegas = chebyshev_weights(maxiter)
        # iterate k in g[k % 4] (a launch reads x_k, x_{k-1} and writes x_{k+1}, x_{k+2}); x_0 = 0
        g = [torch.empty(shape, dtype=D.F64, device=self.dev) for _ in range(4)]
        zero = None
        ring = torch.empty(22 * self.L, dtype=D.F64, device=self.dev)

        def it_ptr(k):
            return None if k == 0 else D.ptr(g[k % 4])

        def launch(k, kk):
            nonlocal zero
            gprev = None
            if k == 1:  # x_0 = 0 as a Chebyshev predecessor (only when the first batch is one sweep)
                if zero is None:
                    zero = torch.zeros(shape, dtype=D.F64, device=self.dev)
                gprev = D.ptr(zero)
            elif k >= 2:
                gprev = D.ptr(g[(k - 1) % 4])
            _lib.check(L.akb_gd_grad_sweeps_f64(
                *self._tri_args(), D.ptr(self.xptr), D.ptr(self.xidx), D.ptr(f), nvals, it_ptr(k), gprev,
                float(omegas[k]), float(omegas[k + 1] if kk == 2 else 1.0), kk, D.ptr(g[(k + 1) % 4]),
                D.ptr(g[(k + 2) % 4]) if kk == 2 else None, D.ptr(ring), D.ptr(change[k:]), s))
        # the first check after 12 sweeps (the C3 hits need ~15 at GRADIENT_TOL), then batches sized
        # from the observed decay rate: each check is a host round trip
        it, batch = 0, (max(check_every, 12) if check_every == 8 else check_every)
        hist = []
        while it < maxiter:
            stop = min(it + batch, maxiter)
            k = it
            while k < stop:
                kk = 2 if stop - k >= 2 else 1
                launch(k, kk)
                k += kk
            if not self._checked:  # the pocket check's word rides on the first batch's copy
                hv = torch.cat([change[it:stop], self._status]).cpu().numpy()
                self._check_status(hv[-1])
                ch = hv[:-1].view(np.float64)
            else:
                ch = change[it:stop].cpu().numpy().view(np.float64)
            done = np.nonzero(ch < tol)[0]
            it = stop
            if done.size:
                hist.extend(ch.tolist())
                break
            # the change decays geometrically: queue about as many sweeps as the observed rate says
            # remain (the host checks once per batch; a batch overshoots by at most one sweep then)
            hist.extend(ch.tolist())
            batch = check_every
            if adaptive and len(hist) >= 4 and hist[-1] > 0 and hist[-4] > hist[-1]:
                rate = (hist[-1] / hist[-4]) ** (1.0 / 3.0)
                need = int(np.ceil(np.log(tol / hist[-1]) / np.log(rate)))
                batch = int(min(max(need, 1), check_every))
        self.sweeps = it
        self.history = hist  # the largest relative change of each sweep's Jacobi step
        if it == 0:
            return torch.zeros(shape, dtype=D.F64, device=self.dev)
        return g[it % 4]

    def interp(self, values, gx, gy, tol=GRADIENT_TOL):
        """(nvals, n) values -> (nvals, len(gy), len(gx)) on the meshgrid of gx x gy."""
        L = _lib.lib()
        f = _dev(values, self.dev).reshape(-1, self.nv * self.nh).contiguous()
        grad = self.gradients(f, tol=tol)
        gx = _dev(gx, self.dev).reshape(-1)
        gy = _dev(gy, self.dev).reshape(-1)
        mx, my = int(gx.numel()), int(gy.numel())
        nvals = int(f.shape[0])
        owner = torch.empty(mx * my, dtype=torch.int32, device=self.dev)
        out = torch.empty((nvals, my, mx), dtype=D.F64, device=self.dev)
        _lib.check(L.akb_gd_eval_f64(*self._tri_args(), D.ptr(gx), mx, D.ptr(gy), my, D.ptr(f), D.ptr(grad), nvals,
                                     D.ptr(owner), D.ptr(out), D.stream_handle()))
        return out

    def interp_cone(self, values, gx, gy, sweeps=CONE_SWEEPS, stream=None):
        """interp with the gradients of exactly `sweeps` Chebyshev sweeps from zero, formed only where
        the targets read them (akb_gd_cone_eval_f64: a patch per interior target cell, the boundary
        band globally). Equal bit for bit to interp on gradients(maxiter=sweeps, tol=0); one launch
        sequence; the first call on a grid reads the pocket check's status word (one host
        synchronisation), and a grid it flagged is refused on every call. self.cone_change: the
        change one more sweep would make at the interior target cells' corners (device, scipy's
        measure as ordered double bits)."""
        L = _lib.lib()
        self._check_status()  # re-raises on every call for a triangulation the pocket check flagged
        f = _dev(values, self.dev).reshape(-1, self.nv * self.nh).contiguous()
        gx = _dev(gx, self.dev).reshape(-1)
        gy = _dev(gy, self.dev).reshape(-1)
        mx, my = int(gx.numel()), int(gy.numel())
        nvals = int(f.shape[0])
        need = int(L.akb_gd_cone_work_bytes(self.nv, self.nh, mx, my, nvals))
        work = torch.empty(need // 8 + 1, dtype=D.F64, device=self.dev)
        owner = torch.empty(mx * my, dtype=torch.int32, device=self.dev)
        out = torch.empty((nvals, my, mx), dtype=D.F64, device=self.dev)
        # [0] the change measure at the interior target cells' corners, [1] the value-error estimate
        self.cone_change = torch.zeros(2, dtype=torch.int64, device=self.dev)
        om = chebyshev_weights(max(int(sweeps), 1))
        _lib.check(L.akb_gd_cone_eval_f64(*self._tri_args(), D.ptr(self.xptr), D.ptr(self.xidx), D.ptr(gx), mx,
                                          D.ptr(gy), my, D.ptr(f), nvals, int(sweeps), D.host_f64(om), D.ptr(work),
                                          D.ptr(owner), D.ptr(out), D.ptr(self.cone_change),
                                          D.stream_handle(stream)))
        self.sweeps = int(sweeps)
        return out


def _axes(grid_H, grid_V):
    gh = np.asarray(grid_H.cpu() if isinstance(grid_H, torch.Tensor) else grid_H, dtype=np.float64)
    gv = np.asarray(grid_V.cpu() if isinstance(grid_V, torch.Tensor) else grid_V, dtype=np.float64)
    if gh.ndim != 2 or gh.shape != gv.shape:
        raise ValueError("xi must be a meshgrid pair (grid_H, grid_V) of equal 2-D shapes")
    gx, gy = gh[0], gv[:, 0]
    if not (np.array_equal(gh, np.broadcast_to(gx, gh.shape)) and np.array_equal(gv, np.broadcast_to(gy[:, None], gv.shape))):
        raise ValueError("xi must be a meshgrid (rows of grid_H equal, columns of grid_V equal)")
    if np.any(np.diff(gx) < 0) or np.any(np.diff(gy) < 0):
        raise ValueError("the target axes must be ascending (np.linspace(min, max, n))")
    return gx, gy


def griddata(points, values, xi, method="cubic", fill_value=np.nan, rescale=False, grid_shape=None):
    """Drop-in for the driver's scipy.interpolate.griddata calls: points = (y, z) of the ray grid's
    hits in ray order, xi = (grid_H, grid_V) from np.meshgrid. The ray grid is taken to have the
    target grid's shape (as the driver builds both from ray_num_V x ray_num_H) unless grid_shape
    = (n_v, n_h) says otherwise. values may be (n,) or (k, n) (k maps on one triangulation).
    numpy in -> numpy out; torch values -> device tensor."""
    if method != "cubic":
        raise NotImplementedError("only method='cubic' (the driver's) runs on the device")
    if not (isinstance(fill_value, float) and np.isnan(fill_value)) or rescale:
        raise NotImplementedError("fill_value=nan, rescale=False only (the driver's)")
    px, py = points
    gx, gy = _axes(*xi)
    nv, nh = grid_shape if grid_shape is not None else (len(gy), len(gx))
    cg = CubicGrid(px, py, nv, nh)
    out = cg.interp(values, gx, gy)
    single = (values.dim() if isinstance(values, torch.Tensor) else np.ndim(values)) == 1
    out = out[0] if single else out
    return out if isinstance(values, torch.Tensor) else out.cpu().numpy()
