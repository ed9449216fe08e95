"""Focus sweeps: the detector-plane searches of the drivers.

find_defocus (AKB_raytrace_20250312.py:9086-9170) traces once and then intersects the same rays
with 50 detector planes per loop, 10 loops, taking np.std of the hits' y and z on each plane and
narrowing the range around the best one. plane_std_sweep does one such loop on the device for any
number of planes at once: one kernel reads each ray once and feeds every plane's hit y / z to
numpy-order leaf sums (the means), a second feeds the squared deviations (np.std's second pass),
so np.std comes out exactly as the reference computes it (the argmin, and find_defocus's answer,
are the reference's own) without writing a row per plane. PlaneSweep(fused=False) keeps the
row-writing variant (akb_plane_sweep_rows_f64 + akb_pairwise_sum_f64) for comparison.
"""
import numpy as np
import torch

from . import _lib
from . import device as D
from .reduce import LeafSink, RowSums


def _dev3(a, dev):
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
    return t.to(device=dev, dtype=D.F64).contiguous()


class PlaneSweep:
    """Rays (dir, pt: (3, n)) held on the device for repeated plane sweeps."""

    def __init__(self, rays, points, subset=None, fused=True):
        self.fused = bool(fused)
        self._sinks = {}
        self.dev = D.device()
        self.dir = _dev3(rays, self.dev)
        self.pt = _dev3(points, self.dev)
        self.n = int(self.dir.shape[1])
        self.subset = None if subset is None else torch.as_tensor(np.asarray(subset, dtype=np.int64)).to(self.dev)
        self.m = self.n if self.subset is None else int(self.subset.shape[0])
        self.sums = RowSums()

    def std(self, plane_j):
        """np.std of the hit y and z on each plane x = -j (coeffs_det[9] = j): two host arrays."""
        L = _lib.lib()
        j = torch.from_numpy(np.ascontiguousarray(plane_j, dtype=np.float64)).to(self.dev)
        P = int(j.shape[0])
        if self.fused:
            sink = self._sinks.get(P)
            if sink is None:
                sink = self._sinks[P] = LeafSink(-(-2 * P // 16) * 16, self.m, 0, self.dev)
            args = (D.ptr(self.dir), D.ptr(self.pt), self.n, self.n, D.ptr(self.subset), self.m, D.ptr(j), P)
            _lib.check(L.akb_plane_sweep_sink_f64(*args, None, sink.desc, D.stream_handle()))
            s1 = sink.finish()[0][:2 * P].clone()
            _lib.check(L.akb_plane_sweep_sink_f64(*args, D.ptr(s1), sink.desc, D.stream_handle()))
            s2 = sink.finish()[0][:2 * P]
            sd = np.sqrt(s2.cpu().numpy() / self.m)  # np.std: ret / rcount, then sqrt
            return sd[0::2], sd[1::2]
        rows = torch.empty((2 * P, self.m), dtype=D.F64, device=self.dev)
        args = (D.ptr(self.dir), D.ptr(self.pt), self.n, self.n, D.ptr(self.subset), self.m, D.ptr(j), P)
        _lib.check(L.akb_plane_sweep_rows_f64(*args, None, D.ptr(rows), D.stream_handle()))
        s1, _ = self.sums(rows)
        _lib.check(L.akb_plane_sweep_rows_f64(*args, D.ptr(s1), D.ptr(rows), D.stream_handle()))
        s2, _ = self.sums(rows)
        var = s2.cpu().numpy() / self.m  # np.std: ret / rcount, then sqrt
        sd = np.sqrt(var)
        return sd[0::2], sd[1::2]


def plane_std_sweep(rays, points, plane_j, subset=None):
    return PlaneSweep(rays, points, subset).std(plane_j)


def find_defocus(rays, points, s2f_middle, defocus, ray_num, sweep=None):
    """Drop-in for find_defocus (:9086): same range, steps, loops and update rule; each loop's 50
    planes in one device sweep. `defocus` and `ray_num` are accepted as the reference's are (they
    only feed its unused per-aperture sizes)."""
    sw = sweep or PlaneSweep(rays, points)
    a_min, a_max = -0.3, 0.3
    shrink, steps = 0.1, 50
    best_a = None
    for _ in range(10):
        a = np.linspace(a_min, a_max, steps)
        j = np.array([-(s2f_middle + a[i]) for i in range(steps)])  # coeffs_det[9] as the reference forms it
        size_h, size_v = sw.std(j)
        best_a = (a[np.argmin(size_h)] + a[np.argmin(size_v)]) / 2
        delta = (a_max - a_min) * shrink
        a_min = best_a - delta / 2
        a_max = best_a + delta / 2
    return best_a
