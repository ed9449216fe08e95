"""Time the leaf-sink finish (k_leaf_chunks + k_pw_final) and the tilt-parameter kernel alone."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from akbraytracing_amd import _lib, device as D
from akbraytracing_amd.reduce import LeafSink

dev = D.device()
L = _lib.lib()
for n in (1221 * 8192, 2137, 10004569):
    sink = LeafSink(5, n, 0b00011, dev)
    sink.buf.zero_()
    for _ in range(3):
        sink.finish()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        sink.finish()
    e1.record()
    torch.cuda.synchronize()
    print(f"finish n={n}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us", flush=True)
s5 = torch.tensor([1e-3, -2e-3, 1.0, 2.0, 3.0], dtype=torch.float64, device=dev) * 1e7
c5 = torch.full((5,), 10 ** 7, dtype=torch.int64, device=dev)
P = torch.empty(23, dtype=torch.float64, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    L.akb_tilt_params_f64(D.ptr(s5), D.ptr(c5), D.ptr(P), None, None, 0, D.stream_handle())
e0.record()
for _ in range(50):
    L.akb_tilt_params_f64(D.ptr(s5), D.ptr(c5), D.ptr(P), None, None, 0, D.stream_handle())
e1.record()
torch.cuda.synchronize()
print(f"tilt params: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us")
