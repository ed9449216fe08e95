"""Sanitizer build of the host code: the library's host-side C++ (akb_host.cpp: the
resample; akb_gd_host.cpp: the pocket triangulation with its fixed-capacity arrays;
akb_affine_host.cpp: contours, polygons and the affine solve of extract_affine_square_region) and the
oracle's C restatement, compiled with -fsanitize=address,undefined into a standalone driver
(tests/sanitize/host_asan_driver.cpp) and run over random, ragged, NaN and degenerate inputs.
GPU code is not sanitized (not available on this pool): the driver links host code only."""
import os
import subprocess

import pytest

from conftest import ROOT

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
CLANG = os.path.join(ROCM, "lib", "llvm", "bin", "clang")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_code_under_asan_and_ubsan(tmp_path):
    csrc = os.path.join(ROOT, "akbraytracing_amd", "csrc")
    exe = str(tmp_path / "host_asan")
    san = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-ffp-contract=off"]
    # the oracle's C with the same clang (one sanitizer runtime in the process)
    oobj = str(tmp_path / "akb_oracle.o")
    r = subprocess.run([CLANG, "-c", "-std=c11", "-fopenmp"] + san + [os.path.join(ROOT, "oracle", "akb_oracle.c"),
                        "-o", oobj], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    objs = [oobj]
    for src in (os.path.join(ROOT, "tests", "sanitize", "host_asan_driver.cpp"), os.path.join(csrc, "akb_host.cpp"),
                os.path.join(csrc, "akb_gd_host.cpp"), os.path.join(csrc, "akb_affine_host.cpp")):
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        r = subprocess.run([HIPCC, "-c", "--offload-arch=gfx950", "-std=c++17", "-fno-gpu-sanitize"] + san +
                           [src, "-o", obj], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        objs.append(obj)
    r = subprocess.run([HIPCC, "-fsanitize=address,undefined", "-fno-gpu-sanitize", "-fopenmp"] + objs + ["-o", exe],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    supp = tmp_path / "lsan.supp"
    supp.write_text("leak:libomp.so\n")  # the OpenMP runtime's own thread-pool allocations
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               LSAN_OPTIONS=f"suppressions={supp}", OMP_NUM_THREADS="2")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "resample:" in r.stdout and "cut corner" in r.stdout and "affine:" in r.stdout
