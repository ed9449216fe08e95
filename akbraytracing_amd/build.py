"""Build libakb_hip.so (the C ABI of include/akb_raytrace.h) for gfx950 with hipcc, in-tree.

    python -m akbraytracing_amd.build

The library is compiled with -ffp-contract=off: the trace kernels depend on every product and
sum being rounded separately, in numpy's order, to reproduce the reference bit for bit.
"""
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
SO = os.path.join(LIBDIR, "libakb_hip.so")
SOURCES = ["akb_trace.hip", "akb_reduce.hip", "akb_huygens.hip", "akb_psf.hip", "akb_psfcalc.hip", "akb_griddata.hip", "akb_focus.hip", "akb_host.cpp",
           "akb_gd_host.cpp", "akb_affine_host.cpp"]
HEADERS = ["akb_common.h", "akb_sincos.h", "akb_pairwise.h", os.path.join("..", "..", "include", "akb_raytrace.h")]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("AKB_OFFLOAD_ARCH", "gfx950")


def sources_hash(csrc=CSRC):
    """sha256 over every compiled source and included header (fixed order, name + bytes). It is
    compiled into the library (akb_sources_hash) and compared by _lib.lib() at load time."""
    h = hashlib.sha256()
    for rel in SOURCES + HEADERS:
        h.update(os.path.basename(rel).encode() + b"\0")
        with open(os.path.join(csrc, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def needs_build():
    if not os.path.exists(SO):
        return True
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    return _newest(deps) > os.path.getmtime(SO)


def build(force=False, verbose=True, out=None, defines=()):
    """Compile each source to an object in parallel (hipcc -c), then link the shared library.
    out / defines: an A/B variant (another path, extra -D flags; loaded through AKB_LIB)."""
    if out is None and not force and not needs_build():
        return SO
    os.makedirs(LIBDIR, exist_ok=True)
    tag = "" if out is None else "_" + os.path.splitext(os.path.basename(out))[0]
    objdir = os.path.join(LIBDIR, "obj" + tag)
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Wall",
             "-Wno-unused-function", f'-DAKB_SOURCES_HASH="{sources_hash()}"'] + [f"-D{d}" for d in defines]
    jobs, objs = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        cmd = [hipcc] + flags + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        jobs.append((src, subprocess.Popen(cmd)))
    failed = [src for src, p in jobs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc -c {' '.join(failed)}")
    target = SO if out is None else out
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", target + ".tmp"] + objs
    cmd += [f"-L{ROCM}/lib", "-lrocfft", f"-Wl,-rpath,{ROCM}/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(SO)
