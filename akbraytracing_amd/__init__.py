"""MI355X-native AKB ray-trace / wavefront / PSF hot path (Kakekakechan/AKBRaytracing).

Modules
  primitives  drop-in mirr_ray_intersection, norm_vector, reflect_ray, normalize_vector,
              plane_ray_intersection, rotate_vectors, rotate_points (one HIP kernel each)
  trace       fused K-mirror chain kernel (device-resident), staged exact path
  wavefront   the 'ray_wave' hot path of plot_result_debug / KB_debug on the device
  reduce      numpy-exact device sums (np.sum / np.mean / np.nanmean order)
  psf         compute_psf_fft on rocFFT (+ batched multi-wavelength psf_stack)
  wavecalc    Huygens-Fresnel propagation (WaveField3D, forward_propagation_*_batch)
  dist        one process per GPU over torch.distributed (RCCL): ray-row / target sharding
  install     rebind a reference module's names to these implementations

Everything runs through libakb_hip.so (include/akb_raytrace.h). No CPU fallback.
"""
import os as _os

import torch as _torch  # noqa: F401  (loads torch's HIP runtime before libakb_hip.so)

from ._lib import AKBError, lib  # noqa: F401
from .install import NATIVE_NAMES, install, uninstall  # noqa: F401

DROPIN_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "dropin")

__all__ = ["install", "uninstall", "NATIVE_NAMES", "lib", "AKBError", "DROPIN_DIR"]
