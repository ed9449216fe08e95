"""griddata(method='cubic') of the 'ray_wave' driver on the device.

The driver interpolates the per-ray DistError2 and Wave2 from the detector hits onto a regular
grid (AKB_raytrace_20250312.py:3673, :3689):

    griddata((detcenter2[1, :], detcenter2[2, :]), Wave2, (grid_H, grid_V), method='cubic')

scipy answers with a Clough-Tocher interpolant on the points' Delaunay triangulation. The points
are the ray grid's hits, a smoothly deformed n_v x n_h lattice, so CubicGrid builds that
triangulation structurally (akb_griddata.hip: cell diagonals by the in-circle test, the hull
pockets on the host, local-Delaunay checks that refuse a grid where this would not be qhull's
answer), estimates the vertex gradients by sweeps of scipy's own local solve until they stop
changing (line Gauss-Seidel in LDS strips: each row sees its upper neighbours' new values), and
evaluates the patches on the device. Agreement with scipy is to rounding on the reference's
65 x 65 run (tests/test_gpu_parity.py), not bit for bit: qhull's co-circular tie-breaks and
scipy's Gauss-Seidel stopping point (1e-6; these sweeps run to 1e-10) are not reproduced.
"""
import numpy as np
import torch

from . import _lib
from . import device as D

_F_NONCONVEX, _F_NOT_DELAUNAY, _F_POCKET, _F_POS, _F_NEG = 1, 2, 4, 8, 16


def _dev(a, dev, dtype=D.F64):
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dtype)


class CubicGrid:
    """The triangulation of an n_v x n_h grid of points (x, y: (n_v * n_h,) row-major), reused for
    any number of value sets and target grids."""

    def __init__(self, x, y, n_v, n_h, delaunay_tol=1e-10):
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
        if not bool(torch.isfinite(self.x).all() & torch.isfinite(self.y).all()):
            raise ValueError("griddata: non-finite point coordinates (a ray that missed)")
        s = D.stream_handle()
        self.diag = torch.empty((self.nv - 1) * (self.nh - 1), dtype=torch.uint8, device=self.dev)
        flags = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.L = 2 * (self.nh - 1) + 2 * (self.nv - 1)
        ring = torch.empty((2, self.L), dtype=D.F64, device=self.dev)
        _lib.check(L.akb_gd_cells_f64(D.ptr(self.x), D.ptr(self.y), self.nv, self.nh, D.ptr(self.diag),
                                      float(delaunay_tol), D.ptr(flags), D.ptr(ring[0]), D.ptr(ring[1]), s))
        rh = ring.cpu().numpy()
        cap = self.L
        tri = np.zeros((cap, 3), np.int32)
        nbr = np.zeros((cap, 3), np.int32)
        edge = np.zeros(self.L, np.int32)
        xptr = np.zeros(self.L + 1, np.int32)
        xidx = np.zeros(6 * cap, np.int32)
        npk = np.zeros(1, np.int32)
        hp = lambda a: a.ctypes.data_as(_lib.c_vp)  # noqa: E731
        _lib.check(L.akb_gd_pockets(hp(np.ascontiguousarray(rh[0])), hp(np.ascontiguousarray(rh[1])), self.nv,
                                    self.nh, cap, hp(npk), hp(tri), hp(nbr), hp(edge), hp(xptr), hp(xidx)))
        self.npock = int(npk[0])
        k = max(self.npock, 1)
        self.ptri = torch.from_numpy(tri[:k].copy()).to(self.dev)
        self.pnbr = torch.from_numpy(nbr[:k].copy()).to(self.dev)
        self.edge_tri = torch.from_numpy(edge).to(self.dev)
        self.xptr = torch.from_numpy(xptr).to(self.dev)
        self.xidx = torch.from_numpy(xidx[:max(int(xptr[-1]), 1)].copy()).to(self.dev)
        _lib.check(L.akb_gd_check_pockets(D.ptr(self.x), D.ptr(self.y), self.nv, self.nh, D.ptr(self.diag),
                                          self.npock, D.ptr(self.ptri), D.ptr(self.pnbr), D.ptr(self.edge_tri),
                                          float(delaunay_tol), D.ptr(flags), s))
        f = int(flags.item())
        if f & _F_NONCONVEX or (f & _F_POS and f & _F_NEG):
            raise _lib.AKBError("griddata: the points do not form a convex, unfolded lattice")
        if f & (_F_NOT_DELAUNAY | _F_POCKET):
            raise _lib.AKBError("griddata: the grid is too distorted for the structured Delaunay triangulation")
        self.sweeps = 0

    def _tri_args(self):
        return (D.ptr(self.x), D.ptr(self.y), self.nv, self.nh, D.ptr(self.diag), self.npock, D.ptr(self.ptri),
                D.ptr(self.pnbr), D.ptr(self.edge_tri))

    def gradients(self, values, tol=1e-10, maxiter=400, check_every=8, adaptive=True):
        """estimate_gradients_2d_global for (nvals, n) values: (nvals, n, 2) device tensor. The sweeps
        stop after the first batch holding one whose largest relative change is below tol; with
        adaptive, batches after the first are sized from the observed decay rate."""
        L = _lib.lib()
        f = _dev(values, self.dev)
        f = f.reshape(-1, self.nv * self.nh).contiguous()
        nvals = int(f.shape[0])
        g = [torch.zeros((nvals, self.nv * self.nh, 2), dtype=D.F64, device=self.dev) for _ in range(2)]
        change = torch.zeros(maxiter, dtype=torch.int64, device=self.dev)
        ring = torch.empty(10 * self.L, dtype=D.F64, device=self.dev)
        s = D.stream_handle()
        cur, it, batch = 0, 0, check_every
        hist = []
        while it < maxiter:
            stop = min(it + batch, maxiter)
            for k in range(it, stop):
                _lib.check(L.akb_gd_grad_sweep_f64(*self._tri_args(), D.ptr(self.xptr), D.ptr(self.xidx), D.ptr(f),
                                                   nvals, D.ptr(g[cur]), D.ptr(g[1 - cur]), D.ptr(ring),
                                                   D.ptr(change[k:]), s))
                cur = 1 - cur
            ch = change[it:stop].cpu().numpy().view(np.float64)
            done = np.nonzero(ch < tol)[0]
            it = stop
            if done.size:
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
        return g[cur]

    def interp(self, values, gx, gy, tol=1e-10):
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
