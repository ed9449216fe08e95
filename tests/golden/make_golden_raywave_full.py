"""Record plot_result_debug(params, 'ray_wave') at the bench's full sizes (build container only;
the reference is read from /root/reference and never travels):

    python tests/golden/make_golden_raywave_full.py [n ...]      (default: 1001 3163)

The live __main__ path (AKB_raytrace_20250312.py:14586-14611, option_set=True) on an n x n ray grid
(n = 3163 is BASELINE configs[2], 1e7 rays). The run is stopped at its second griddata call
(:3689), once both gridding inputs exist. Recorded per n, on a seeded sample of rays (the resample
picks plus 8192 rays drawn over the whole grid), straight from the reference's own calls:

  n{n}_idx              sampled ray indices (flat iv * n + ih)
  n{n}_last_hit         pass 2's hit on mirror 4 (the 8th mirr_ray_intersection of n^2 rays)
  n{n}_dir_out          pass 2's exit direction (the 8th reflect_ray of n^2 rays)
  n{n}_det2             detcenter2 rows y, z (the griddata points, :3673 / :3689)
  n{n}_dist_err2        DistError2 (griddata values of :3673)
  n{n}_wave2            Wave2 (griddata values of :3689)
  n{n}_stats            nanmean / nanstd of DistError2 and Wave2 over all n^2 rays, min / max of
                        detcenter2 y and z (the grid extent, :3654-3657)

and the reference's gridding step with the bench's 128 x 128 pupil grid in place of the driver's
n x n one (scipy griddata(cubic) of both value sets on one Delaunay triangulation of the n^2 points,
matrixWave2 minus its nanmean, then the reference's own plane_correction_with_nan_and_outlier_filter,
:3654-3696, :9630-9693):

  n{n}_gx, n{n}_gy      the grid axes (np.linspace of the extents, 128 points)
  n{n}_map_dist, n{n}_map_wave              griddata outputs (matrixWave2 after the nanmean removal)
  n{n}_map_dist_c, n{n}_map_wave_c          the plane-corrected maps
  n{n}_qhull_flips      cells whose diagonal in qhull's triangulation is not the exact in-circle
                        choice (near-cocircular cells: qhull's roundoff model, on coordinates
                        ~2 cm from the origin, merges facets whose in-circle margin is ~1e-6 of
                        the cell's scale and triangulates them its own way)
  n{n}_ambiguous        (128, 128) targets whose containing cell lies within AMBIG_CELLS cells of
                        such a cell: there scipy's answer depends on qhull's pick (the estimated
                        gradients carry a flip's effect a few cells, ~1/2 per cell)

Uses make_golden's stand-ins (numba, cv2, tifffile). scipy's qhull at 3163^2 needs ~10 GB and
several minutes.
"""
import contextlib
import io
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as MG  # noqa: E402

GRID = 128
NSAMPLE = 8192
AMBIG_CELLS = 10


class SampleRecorder:
    """Keeps only the sampled columns of the reference's full-grid primitive calls."""

    NAMES = ("mirr_ray_intersection", "reflect_ray")

    def __init__(self, mod, N, idx):
        self.mod, self.N, self.idx = mod, N, idx
        self.out = {n: [] for n in self.NAMES}
        self.orig = {n: getattr(mod, n) for n in self.NAMES}
        for n in self.NAMES:
            setattr(mod, n, self._wrap(n, self.orig[n]))

    def _wrap(self, name, f):
        def g(*a, **k):
            r = f(*a, **k)
            arr = np.asarray(r)
            if arr.ndim == 2 and arr.shape[1] == self.N:
                self.out[name].append(np.array(arr[:, self.idx]))
            return r
        return g

    def restore(self):
        for n, f in self.orig.items():
            setattr(self.mod, n, f)


def sample_idx(n):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import oracle.pipeline as OPL
    _, v_idx, _, _, h_idx = OPL.sample_indices(n, n)
    rng = np.random.default_rng(n)
    return np.unique(np.concatenate([h_idx, v_idx, rng.integers(0, n * n, NSAMPLE), [0, n - 1, n * n - n, n * n - 1]]))


def qhull_ambiguity(tri, y, z, n, GH, GV):
    """(flipped cells (n-1, n-1), ambiguous targets GH.shape): cells whose qhull diagonal is not the
    exact in-circle choice of akb_griddata.hip's k_gd_cells (same expression, same operation order),
    and the targets within AMBIG_CELLS cells of one."""
    from scipy.ndimage import binary_dilation
    S = np.sort(tri.simplices, axis=1).astype(np.int64)
    a, b, c = S[:, 0], S[:, 1], S[:, 2]
    qd = np.full((n - 1) * (n - 1), -1, np.int8)

    def mark(sel, cell_vertex, d):
        iv, ih = np.divmod(cell_vertex[sel], n)
        ok = (iv < n - 1) & (ih < n - 1)
        qd[(iv * (n - 1) + ih)[ok]] = d

    mark((b == a + 1) & (c == a + n + 1), a, 0)
    mark((b == a + n) & (c == a + n + 1), a, 0)
    mark((b == a + 1) & (c == a + n), a, 1)
    mark((b == a + n - 1) & (c == a + n), a - 1, 1)
    Y, Z = y.reshape(n, n), z.reshape(n, n)
    x0, y0 = Y[:-1, :-1], Z[:-1, :-1]
    bx, by = Y[:-1, 1:] - x0, Z[:-1, 1:] - y0
    cx, cy = Y[1:, 1:] - x0, Z[1:, 1:] - y0
    dx, dy = Y[1:, :-1] - x0, Z[1:, :-1] - y0
    adx, ady, bdx, bdy, cdx, cdy = -dx, -dy, bx - dx, by - dy, cx - dx, cy - dy
    A, B, C = adx * adx + ady * ady, bdx * bdx + bdy * bdy, cdx * cdx + cdy * cdy
    det = adx * (bdy * C - B * cdy) - ady * (bdx * C - B * cdx) + A * (bdx * cdy - bdy * cdx)
    o = bx * cy - by * cx
    exact = (np.where(o > 0, det, -det) > 0).astype(np.int8).ravel()
    flips = (qd != exact).reshape(n - 1, n - 1)  # includes cells qhull split some other way (qd = -1)
    near = binary_dilation(flips, iterations=AMBIG_CELLS)
    s = tri.find_simplex(np.stack([GH.ravel(), GV.ravel()], axis=1))
    amb = np.zeros(s.shape, bool)
    inside = s >= 0
    iv, ih = np.divmod(tri.simplices[s[inside]].min(axis=1), n)
    amb[inside] = near[np.minimum(iv, n - 2), np.minimum(ih, n - 2)]
    return flips, amb.reshape(GH.shape)


def record(A, n):
    from scipy.interpolate import CloughTocher2DInterpolator
    from scipy.spatial import Delaunay
    N = n * n
    idx = sample_idx(n)
    A.wave_num_H = A.wave_num_V = n
    A.option_set = True
    rec = SampleRecorder(A, N, idx)
    grid_calls = []
    orig_grid = A.griddata

    def griddata(points, values, xi, method="linear", **kw):
        grid_calls.append((np.array(points[0]), np.array(points[1]), np.array(values)))
        if len(grid_calls) == 2:
            raise StopIteration  # both gridding inputs recorded (:3673, :3689)
        return np.zeros(np.shape(xi[0]))  # the driver's n x n map is not needed before the stop

    A.griddata = griddata
    t0 = time.time()
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            A.plot_result_debug(MG.best_params(), "ray_wave", option_save=False)
    except StopIteration:
        pass
    finally:
        A.griddata = orig_grid
        rec.restore()
    print(f"n={n}: reference trace {time.time() - t0:.1f} s", flush=True)
    isects, refl = rec.out["mirr_ray_intersection"], rec.out["reflect_ray"]
    assert len(isects) == 8 and len(refl) == 8, (len(isects), len(refl))
    (y, z, dist_err2), (y2, z2, wave2) = grid_calls
    assert np.array_equal(y, y2) and np.array_equal(z, z2)
    out = {
        f"n{n}_idx": idx, f"n{n}_last_hit": isects[7], f"n{n}_dir_out": refl[7],
        f"n{n}_det2": np.stack([y[idx], z[idx]]), f"n{n}_dist_err2": dist_err2[idx], f"n{n}_wave2": wave2[idx],
        f"n{n}_stats": np.array([np.nanmean(dist_err2), np.nanstd(dist_err2), np.nanmean(wave2), np.nanstd(wave2),
                                 y.min(), y.max(), z.min(), z.max()]),
    }
    # the gridding step (:3654-3696) onto the bench's 128 x 128 pupil grid
    gx = np.linspace(y.min(), y.max(), GRID)
    gy = np.linspace(z.min(), z.max(), GRID)
    GH, GV = np.meshgrid(gx, gy)
    t0 = time.time()
    tri = Delaunay(np.stack([y, z], axis=1))
    print(f"n={n}: qhull {time.time() - t0:.1f} s", flush=True)
    t0 = time.time()
    m_dist = CloughTocher2DInterpolator(tri, dist_err2)((GH, GV))
    m_wave = CloughTocher2DInterpolator(tri, wave2)((GH, GV))
    print(f"n={n}: Clough-Tocher {time.time() - t0:.1f} s", flush=True)
    flips, amb = qhull_ambiguity(tri, y, z, n, GH, GV)
    print(f"n={n}: {flips.sum()} cells with qhull's other diagonal, {amb.sum()} ambiguous targets", flush=True)
    del tri
    m_wave = m_wave - np.nanmean(m_wave)
    out.update({f"n{n}_qhull_flips": np.int64(flips.sum()), f"n{n}_ambiguous": amb})
    out.update({f"n{n}_gx": gx, f"n{n}_gy": gy, f"n{n}_map_dist": m_dist, f"n{n}_map_wave": m_wave,
                f"n{n}_map_wave_c": A.plane_correction_with_nan_and_outlier_filter(m_wave),
                f"n{n}_map_dist_c": A.plane_correction_with_nan_and_outlier_filter(m_dist)})
    return out


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [1001, 3163]
    MG._stub_modules()
    sys.modules["tifffile"].imwrite = lambda *a, **kw: None
    sys.path.insert(0, MG.REF)
    os.chdir(tempfile.mkdtemp(prefix="akb_golden_full_"))
    import AKB_raytrace_20250312 as A
    import scipy
    path = os.path.join(MG.OUT, "akb_raywave_full.npz")
    out = dict(np.load(path)) if os.path.exists(path) else {}
    out["meta_versions"] = np.array([np.__version__, scipy.__version__])
    for n in sizes:
        out.update(record(A, n))
        np.savez_compressed(path, **out)
        print(f"n={n}: written", flush=True)


if __name__ == "__main__":
    main()
