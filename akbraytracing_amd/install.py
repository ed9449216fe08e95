"""Rebind a reference module's hot-path functions to the GPU implementations.

The reference's drivers resolve their primitives through module globals at call time
(plot_result_debug, KB_debug, ell.calc_reflect, PlanePoints all call
mirr_ray_intersection / norm_vector / reflect_ray / plane_ray_intersection / normalize_vector /
rotate_vectors / rotate_points / compute_psf_fft by name), so rebinding those names after
import redirects every call site without editing the reference:

    import AKB_raytrace_20250312 as A
    import akbraytracing_amd
    akbraytracing_amd.install(A)
    A.plot_result_debug(params, 'ray_wave')      # traces on the MI355X

Wavecalc scripts: install(W) rebinds forward_propagation_numpy_batch /
forward_propagation_cupy_batch(_multi_gpu), used by their WaveField3D.forward_propagation.

The wrappers read the module's live `option_mpmath` flag (AKB_raytrace_20250312.py:92) at call
time and hand the call to the original function when it is set (the mpmath branch, :399-443).
"""
from . import primitives as _P
from . import psf as _psf
from . import wavecalc as _W

_NATIVE = {
    "mirr_ray_intersection": _P.mirr_ray_intersection,
    "norm_vector": _P.norm_vector,
    "reflect_ray": _P.reflect_ray,
    "normalize_vector": _P.normalize_vector,
    "plane_ray_intersection": _P.plane_ray_intersection,
    "rotate_vectors": _P.rotate_vectors,
    "rotate_points": _P.rotate_points,
    "compute_psf_fft": _psf.compute_psf_fft,
    "forward_propagation_numpy_batch": _W.forward_propagation_numpy_batch,
    "forward_propagation_cupy_batch": _W.forward_propagation_cupy_batch,
    "forward_propagation_cupy_batch_multi_gpu": _W.forward_propagation_cupy_batch_multi_gpu,
}
# functions with an mpmath branch in the reference
_MPMATH_AWARE = {"mirr_ray_intersection", "reflect_ray"}


def _wrap(mod, name, original, native):
    def wrapper(*args, **kwargs):
        if name in _MPMATH_AWARE and getattr(mod, "option_mpmath", False):
            return original(*args, **kwargs)
        return native(*args, **kwargs)
    wrapper.__name__ = name
    wrapper.__wrapped__ = original
    wrapper.__akb_native__ = True
    return wrapper


def install(mod, names=None):
    """Rebind `names` (default: every hot-path name the module defines) in `mod`.
    Returns the list of rebound names. uninstall(mod) restores the originals."""
    done = []
    for name in (names or _NATIVE):
        if name not in _NATIVE or not hasattr(mod, name):
            continue
        cur = getattr(mod, name)
        if getattr(cur, "__akb_native__", False):
            done.append(name)
            continue
        setattr(mod, name, _wrap(mod, name, cur, _NATIVE[name]))
        done.append(name)
    return done


def uninstall(mod):
    for name in _NATIVE:
        cur = getattr(mod, name, None)
        if cur is not None and getattr(cur, "__akb_native__", False):
            setattr(mod, name, cur.__wrapped__)
