"""Device plumbing: torch owns device memory and streams; the HIP library gets raw pointers.

All hot-path data is float64 struct-of-arrays, (3, N) row-major, like the reference's arrays.
"""
import atexit
import ctypes
import threading
import time

import numpy as np
import torch

from . import _lib

F64 = torch.float64


def require_gpu():
    if not torch.cuda.is_available():
        raise _lib.AKBError("no HIP device visible: the AKB hot path runs on MI355X only (no CPU fallback)")


def device():
    require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


def stream_handle(stream=None):
    """hipStream_t of a torch stream (default: the current one); a handle passes through."""
    if isinstance(stream, ctypes.c_void_p):
        return stream
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def reserved_stream(reserve, dev=None):
    """A torch stream whose kernels leave `reserve` CUs (a multiple of 8, the same number on every
    XCD) to the device's other streams (akb_stream_create_reserved). The trace's passes run on it
    so the faithful chain's single-workgroup kernels on the back stream start on a free CU instead
    of waiting for one to drain of pass workgroups. It lives until the library unloads: tensors
    freed during the interpreter's teardown may still record events on it."""
    require_gpu()
    dev = dev if dev is not None else device()
    L = _lib.lib()
    sp = ctypes.c_void_p()
    _lib.check(L.akb_stream_create_reserved(int(reserve), ctypes.byref(sp)))
    atexit.register(_quiesce_reserved, dev)
    return torch.cuda.ExternalStream(sp.value, device=dev)


def _quiesce_reserved(dev):
    try:
        torch.cuda.synchronize(dev)
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
    except Exception:  # exit path: never mask the process's own status
        pass


def ptr(t):
    """Raw device pointer of a tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def to_dev(a, dev=None):
    """numpy / torch array -> contiguous float64 device tensor."""
    dev = dev or device()
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=F64).contiguous()
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return torch.from_numpy(arr).to(dev, non_blocking=False)


def host_f64(values):
    """ctypes double array on the host (coefficients, matrices, small vectors)."""
    vals = [float(v) for v in values]
    return (ctypes.c_double * len(vals))(*vals)


def empty(shape, dev=None):
    return torch.empty(shape, dtype=F64, device=dev or device())


def flags_tensor(dev=None):
    return torch.zeros(1, dtype=torch.int32, device=dev or device())


# ---- host wait clock: wall time the issuing (main) thread spends blocked on the device or on a
# worker (events not yet reached, the pocket job), so a caller can tell its own issue cost from its
# waits (bench.py: host_issue_ms_per_step = host_wait_ms_per_step + the pure issue time)
_HOST_WAIT = [0.0]


def host_wait_s():
    """Seconds the main thread has spent in wait_event / wait_result so far."""
    return _HOST_WAIT[0]


def _clock(t0):
    if threading.current_thread() is threading.main_thread():
        _HOST_WAIT[0] += time.perf_counter() - t0


def wait_event(ev):
    """ev.synchronize(), its blocked time on the host wait clock (nothing when ev has passed)."""
    if ev.query():
        return
    t0 = time.perf_counter()
    ev.synchronize()
    _clock(t0)


def wait_result(fut):
    """fut.result(), its blocked time on the host wait clock."""
    if fut.done():
        return fut.result()
    t0 = time.perf_counter()
    try:
        return fut.result()
    finally:
        _clock(t0)
