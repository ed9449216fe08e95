"""Huygens-Fresnel field propagation between sampled surfaces (the Wavecalc_raytrace_fromData
scripts), on the HIP kernel akb_huygens_f64.

  u[i] = sum_j (u_j dS_j) exp(-i k r_ij) / r_ij

Reference API kept (Wavecalc_raytrace_fromData_CPU0402.py:17-124, ..._GPU0402.py:17-201,
..._GPU0402_multi.py:64-229):
  WaveField3D(num, _lambda, wave_num_H, wave_num_V) with .setdata(data), .set_ds(ds),
      .forward_propagation(u_back, num_cores=None)
  forward_propagation_numpy_batch(x, y, z, ubx, uby, ubz, ubu, k, ds, num_cores=None)
  forward_propagation_cupy_batch(x, y, z, ubx, uby, ubz, ubu, k, ds)
  forward_propagation_cupy_batch_multi_gpu(x, y, z, ubx, uby, ubz, ubu, k, ds, devices=None)
Inputs may be numpy arrays or torch tensors; the returned field is a numpy complex128 array
(device tensors in, device tensor out). There is no B x M materialisation and no batching by
free memory: the kernel streams source tiles through LDS (see csrc/akb_huygens.hip).
"""
import threading
import time

import numpy as np
import torch

from . import _lib
from . import device as D


def _field_dev(u, dev):
    if isinstance(u, torch.Tensor):
        return u.to(device=dev, dtype=torch.complex128).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(u, dtype=np.complex128))).to(dev)


# the split partials' scratch (up to ~516 MiB), reused across calls: one per host thread and
# device - the _multi pattern's threads may share a device, and one call queues three kernels
# (the pair sum and the two reduce levels) that must not interleave with another thread's on it
_WORK = threading.local()


def splits_for(n, m):
    """The source-split count the library picks for n targets and m sources (on this device)."""
    return int(_lib.lib().akb_huygens_splits(int(n), int(m)))


def propagate(tx, ty, tz, sx, sy, sz, u_ds, k, stream=None, work=None, splits=0):
    """Device API: all arguments float64 / complex128 device tensors (u_ds already times dS).
    splits: the source-split count (0: the library's for these sizes; a target-sharded caller
    passes splits_for(whole target count, m) so every target's sum is the unsharded one, bit for
    bit). Returns the (N,) complex128 device tensor of target fields."""
    L = _lib.lib()
    dev = tx.device
    n, m = int(tx.shape[0]), int(sx.shape[0])
    out = torch.empty(n, dtype=torch.complex128, device=dev)
    need = int(L.akb_huygens_work_bytes(n, m, int(splits)))
    if need > 0 and (work is None or work.numel() * 8 < need):
        # keyed by (device, stream): calls on two streams of one thread may overlap on the device,
        # so they must not share the split partials
        cache = _WORK.__dict__.setdefault("by_stream", {})
        key = (dev, D.stream_handle(stream).value)
        work = cache.get(key)
        if work is None or work.numel() * 8 < need:
            work = cache[key] = torch.empty(need // 8 + 1, dtype=D.F64, device=dev)
    ur = torch.view_as_real(u_ds)
    _lib.check(L.akb_huygens_f64(D.ptr(tx), D.ptr(ty), D.ptr(tz), n, D.ptr(sx), D.ptr(sy), D.ptr(sz), D.ptr(ur), m,
                                 float(k), D.ptr(torch.view_as_real(out)), int(splits),
                                 D.ptr(work) if need > 0 else None, D.stream_handle(stream)))
    return out


def scale_field(u, ds):
    """u * ds (complex * real, Wavecalc_raytrace_fromData_CPU0402.py:102) on the device."""
    L = _lib.lib()
    out = torch.empty_like(u)
    m = int(u.shape[0])
    _lib.check(L.akb_scale_field_f64(D.ptr(torch.view_as_real(u)), D.ptr(ds), m, D.ptr(torch.view_as_real(out)),
                                     D.stream_handle()))
    return out


def _prepare(x, y, z, ubx, uby, ubz, ubu, ds, dev):
    as_torch = any(isinstance(a, torch.Tensor) for a in (x, ubu))
    tx, ty, tz = (D.to_dev(a, dev) for a in (x, y, z))
    sx, sy, sz = (D.to_dev(a, dev) for a in (ubx, uby, ubz))
    u = _field_dev(ubu, dev)
    d = D.to_dev(ds, dev)
    return as_torch, tx, ty, tz, sx, sy, sz, scale_field(u, d)


def forward_propagation_numpy_batch(x, y, z, u_back_x, u_back_y, u_back_z, u_back_u, k, ds, num_cores=None):
    """Same contract as the CPU script's function (CPU0402.py:87-124); runs on the GPU.
    num_cores is accepted for signature compatibility and ignored."""
    dev = D.device()
    as_torch, tx, ty, tz, sx, sy, sz, u = _prepare(x, y, z, u_back_x, u_back_y, u_back_z, u_back_u, ds, dev)
    out = propagate(tx, ty, tz, sx, sy, sz, u, k)
    return out if as_torch else out.cpu().numpy()


forward_propagation_cupy_batch = forward_propagation_numpy_batch


def forward_propagation_cupy_batch_multi_gpu(x, y, z, u_back_x, u_back_y, u_back_z, u_back_u, k, ds, devices=None):
    """Target sharding over the visible GPUs of this process, one host thread per device
    (the pattern of GPU0402_multi.py:123-229): targets are split into contiguous pieces
    (np.array_split order), sources are replicated, results concatenated in order."""
    D.require_gpu()
    devs = list(range(torch.cuda.device_count())) if devices is None else list(devices)
    x_np = [np.asarray(a.cpu() if isinstance(a, torch.Tensor) else a, dtype=np.float64) for a in (x, y, z)]
    pieces = [np.array_split(a, len(devs)) for a in x_np]
    results = [None] * len(devs)
    errors = []
    # every piece sums its sources in the whole problem's split order: the concatenated field is
    # the one-device field bit for bit
    with torch.cuda.device(devs[0]):
        splits = splits_for(x_np[0].shape[0], np.shape(u_back_u)[0])

    def work(i, dev_id):
        try:
            with torch.cuda.device(dev_id):
                dev = torch.device("cuda", dev_id)
                _, tx, ty, tz, sx, sy, sz, u = _prepare(pieces[0][i], pieces[1][i], pieces[2][i], u_back_x,
                                                        u_back_y, u_back_z, u_back_u, ds, dev)
                results[i] = propagate(tx, ty, tz, sx, sy, sz, u, k, splits=splits).cpu().numpy()
        except Exception as e:  # surfaced after join
            errors.append(e)

    threads = [threading.Thread(target=work, args=(i, d)) for i, d in enumerate(devs)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return np.concatenate(results)


class WaveField3D:
    """Sampled complex field on a surface (CPU0402.py:17-52): coordinates x, y, z, area
    elements ds and the field u, all float64 / complex128."""

    def __init__(self, num, _lambda, wave_num_H, wave_num_V):
        self.u = np.zeros(num, dtype=np.complex128)
        self.x = np.zeros(num, dtype=np.float64)
        self.y = np.zeros(num, dtype=np.float64)
        self.z = np.zeros(num, dtype=np.float64)
        self.lambda_ = np.float64(_lambda)
        self.wave_num_H = wave_num_H
        self.wave_num_V = wave_num_V
        self.ds = None
        self.elapsed = None

    def setdata(self, data):
        self.x = np.array(data[0, :], dtype=np.float64)
        self.y = np.array(data[1, :], dtype=np.float64)
        self.z = np.array(data[2, :], dtype=np.float64)

    def set_ds(self, data):
        self.ds = np.array(data, dtype=np.float64)

    def forward_propagation(self, u_back, num_cores=None):
        """Propagate u_back (a WaveField3D with ds set) onto this surface's points."""
        k = 2.0 * np.pi / self.lambda_
        t0 = time.time()
        self.u = forward_propagation_numpy_batch(self.x, self.y, self.z, u_back.x, u_back.y, u_back.z, u_back.u, k,
                                                 u_back.ds, num_cores=num_cores)
        self.elapsed = time.time() - t0
        print(f"forward_propagation: {self.elapsed:.6f} s")
