"""The device tilt matrices' sin / cos (akb_sincos.h), built for the host with gcc and checked
against correctly rounded values from mpmath (200-bit): the header is shared code, so this pins
the arithmetic the GPU runs (the GPU test compares the device parameter block with the same)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SRC = r'''
#include "akb_sincos.h"
extern "C" void sincos_batch(const double* x, long n, double* s, double* c) {
    for (long i = 0; i < n; ++i) akb_sc::sincos_cr(x[i], s + i, c + i);
}
'''


@pytest.fixture(scope="module")
def sincos_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("sincos")
    cpp = d / "sc.cpp"
    cpp.write_text(SRC)
    so = d / "libsc.so"
    inc = os.path.join(ROOT, "akbraytracing_amd", "csrc")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-I", inc, str(cpp), "-o", str(so)],
                   check=True)
    L = ctypes.CDLL(str(so))
    L.sincos_batch.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]

    def f(x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        s, c = np.empty_like(x), np.empty_like(x)
        L.sincos_batch(x.ctypes.data, x.shape[0], s.ctypes.data, c.ctypes.data)
        return s, c
    return f


def _cr(x):
    import mpmath
    mpmath.mp.prec = 200
    s = np.array([float(mpmath.sin(mpmath.mpf(float(v)))) for v in x])
    c = np.array([float(mpmath.cos(mpmath.mpf(float(v)))) for v in x])
    return s, c


def test_sincos_is_correctly_rounded(sincos_lib):
    pytest.importorskip("mpmath")
    rng = np.random.default_rng(7)
    small = rng.uniform(-1, 1, 6000) * 10.0 ** rng.uniform(-9, 0, 6000) * 0.785  # tilt-angle range
    mid = rng.uniform(-60.0, 60.0, 3000)
    x = np.concatenate([small, mid, [0.0, -0.0, 1e-30, -2e-9, 0.7853981633974483, 1.5707963267948966]])
    s, c = sincos_lib(x)
    rs, rc = _cr(x)
    assert np.array_equal(s, rs) and np.array_equal(c, rc)
    assert np.signbit(s[np.where(x == 0)[0][1]])  # sin(-0) = -0


def test_sincos_nonfinite_and_huge(sincos_lib):
    s, c = sincos_lib(np.array([np.nan, np.inf, 1e300]))
    assert np.isnan(s[0]) and np.isnan(c[0]) and np.isnan(s[1]) and np.isnan(c[1])
    assert s[2] == np.sin(1e300) and c[2] == np.cos(1e300)
