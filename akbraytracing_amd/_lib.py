"""ctypes binding of libakb_hip.so (declarations mirror include/akb_raytrace.h one for one).

The library is loaded lazily on first use. torch is imported first so the process uses torch's
HIP runtime (libamdhip64.so.7 is matched by SONAME), which keeps the device pointers and stream
handles that torch hands us valid inside the library.
"""
import atexit
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from . import build as _build

_LIB = None

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
c_vp = ctypes.c_void_p
MAX_MIRRORS = 7
ABI_VERSION = 17

FLAG_MISS = 0x1
FLAG_ZERO_NORMAL = 0x2
FLAG_ZERO_REFLECT = 0x4
FLAG_ZERO_DIR = 0x8
FLAG_CHAIN_DIR = 1 << 28

# every symbol the header declares (tests check the library exports all of them)
EXPORTS = [
    "akb_last_error", "akb_abi_version", "akb_sources_hash", "akb_device_count",
    "akb_stream_create_reserved", "akb_stream_destroy", "akb_reserved_cu_mask",
    "akb_isect_f64", "akb_normal_f64", "akb_reflect_f64", "akb_normalize_f64", "akb_plane_isect_f64",
    "akb_seglen_f64", "akb_rotate_f64", "akb_fill_nan_f64",
    "akb_trace_chain_f64", "akb_chain_desc_size", "akb_tilt_opd_f64", "akb_tilt_params_f64",
    "akb_tilt_opd_dev_f64", "akb_chain_tilt_f64", "akb_chain_tilt_opd_f64", "akb_trace_chain_samples_f64", "akb_opd_f64", "akb_resample_f64", "akb_plane_sweep_rows_f64",
    "akb_plane_sweep_sink_f64",
    "akb_calc_ds_f64",
    "akb_pairwise_work_bytes", "akb_pairwise_sum_f64", "akb_pupil_sample_f64",
    "akb_leaf_sink_bytes", "akb_leaf_sink_layout", "akb_leaf_finish_work_bytes", "akb_leaf_finish_f64",
    "akb_leaf_parts_f64", "akb_parts_chain_f64",
    "akb_huygens_splits", "akb_huygens_work_bytes", "akb_huygens_f64", "akb_scale_field_f64",
    "akb_psf_work_bytes", "akb_psf_f64", "akb_psf_release_plans", "akb_release_all", "akb_selftest_arith_f64",
    "akb_first_valid_rows_f64", "akb_rotate_work_bytes", "akb_rotate_with_nan_f64", "akb_pupil_post_f64", "akb_pupil_post_work_bytes",
    "akb_moments_work_bytes", "akb_map_moments_f64", "akb_plane_subtract_f64", "akb_legendre_rows_f64",
    "akb_gd_cells_f64", "akb_gd_pockets", "akb_gd_check_pockets", "akb_gd_grad_sweeps_f64",
    "akb_gd_eval_f64", "akb_gd_cone_work_bytes", "akb_gd_patch_timing", "akb_gd_patch_times", "akb_gd_band_times", "akb_gd_patch_phases", "akb_gd_patch_order", "akb_gd_cone_eval_f64", "akb_gd_axes_f64",
    "akb_gd_cells_claims_f64", "akb_gd_claim_pockets_f64", "akb_gd_cone_solve_f64",
    "akb_gd_claims_f64", "akb_gd_cone_part_f64", "akb_gd_part_finish_f64", "akb_gd_ring_f64", "akb_gd_cells_window_f64",
    "akb_trace_chain_batch_f64", "akb_focus_eval_work_bytes", "akb_focus_eval_f64", "akb_sep_search_f64",
    "akb_finish_params_work_bytes", "akb_finish_tilt_params_f64",
    "akb_valid_mask_u8", "akb_external_contours", "akb_approx_poly_dp", "akb_affine_from_points",
    "akb_affine_invert", "akb_warp_affine_f64",
]


class LeafSink(ctypes.Structure):
    """akb_leaf_sink"""
    _fields_ = [
        ("leaf_sum", c_vp), ("leaf_cnt", c_vp), ("tail", c_vp),
        ("nq", c_i32), ("nan_mask", c_i32), ("n", c_i64),
    ]


class ChainDesc(ctypes.Structure):
    """akb_chain_desc"""
    _fields_ = [
        ("n_mirrors", c_i32),
        ("negative", c_i32 * MAX_MIRRORS),
        ("coeffs", (c_dbl * 10) * MAX_MIRRORS),
        ("det_ghij", c_dbl * 4),
        ("dir", c_vp), ("dir_ld", c_i64), ("dir_inc", c_i64),
        ("tan_h", c_vp), ("tan_v", c_vp), ("n_h", c_i64), ("n_v", c_i64),
        ("ray0", c_i64),
        ("n_rays", c_i64),
        ("org", c_vp), ("org_ld", c_i64), ("org_inc", c_i64),
        ("src", c_dbl * 3),
        ("hits", c_vp), ("hits_ld", c_i64),
        ("last_hit", c_vp), ("last_hit_ld", c_i64),
        ("dir_out", c_vp), ("dir_out_ld", c_i64),
        ("det_out", c_vp), ("det_out_ld", c_i64),
        ("opl", c_vp),
        ("atan_h", c_vp), ("atan_v", c_vp),
        ("samp_h_begin", c_i64), ("samp_h_end", c_i64),
        ("samp_v_col", c_i64),
        ("samp_h", c_vp), ("samp_v", c_vp),
        ("flags", c_vp),
        ("sink", LeafSink),
        ("pert_h", c_vp), ("pert_v", c_vp), ("pert_terms", c_i32),
        ("copy_src", c_vp), ("copy_dst", c_vp), ("copy_n", c_i64),
    ]


class AKBError(RuntimeError):
    pass


def _declare(L):
    v3 = [c_vp, c_i64, c_i64]
    sig = {
        "akb_last_error": ([], ctypes.c_char_p),
        "akb_abi_version": ([], c_int),
        "akb_sources_hash": ([], ctypes.c_char_p),
        "akb_device_count": ([], c_int),
        "akb_stream_create_reserved": ([c_int, c_vp], c_int),
        "akb_stream_destroy": ([c_vp], c_int),
        "akb_reserved_cu_mask": ([c_int, c_int, c_vp], c_int),
        "akb_isect_f64": ([c_vp] + v3 + v3 + [c_int, c_i64, c_vp, c_i64, c_vp, c_vp], c_int),
        "akb_normal_f64": ([c_vp] + v3 + [c_i64, c_vp, c_i64, c_int, c_vp, c_vp], c_int),
        "akb_reflect_f64": (v3 + v3 + [c_i64, c_vp, c_i64, c_int, c_vp, c_vp], c_int),
        "akb_normalize_f64": (v3 + [c_i64, c_vp, c_i64, c_vp, c_vp], c_int),
        "akb_plane_isect_f64": ([c_vp] + v3 + v3 + [c_i64, c_vp, c_i64, c_vp], c_int),
        "akb_seglen_f64": (v3 + v3 + [c_i64, c_vp, c_vp], c_int),
        "akb_rotate_f64": ([c_vp, c_vp, c_vp] + v3 + [c_i64, c_vp, c_i64, c_vp], c_int),
        "akb_fill_nan_f64": ([c_vp, c_i64, c_int, c_i64, c_vp], c_int),
        "akb_trace_chain_f64": ([ctypes.POINTER(ChainDesc), c_vp], c_int),
        "akb_chain_desc_size": ([], c_i64),
        "akb_tilt_opd_f64": ([c_vp] * 5 + [c_vp, c_vp, c_vp, c_i64, c_i64] + [c_vp] * 6
                             + [ctypes.POINTER(LeafSink), c_vp], c_int),
        "akb_tilt_params_f64": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp], c_int),
        "akb_finish_params_work_bytes": ([ctypes.POINTER(LeafSink)], c_i64),
        "akb_finish_tilt_params_f64": ([ctypes.POINTER(LeafSink)] + [c_vp] * 5 + [c_int] + [c_vp] * 2, c_int),
        "akb_tilt_opd_dev_f64": ([c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64] + [c_vp] * 6
                                 + [ctypes.POINTER(LeafSink), c_vp], c_int),
        "akb_trace_chain_samples_f64": ([ctypes.POINTER(ChainDesc), c_vp], c_int),
        "akb_trace_chain_batch_f64": ([ctypes.POINTER(ChainDesc), c_int, c_vp], c_int),
        "akb_focus_eval_work_bytes": ([c_int, c_int, c_i64], c_i64),
        "akb_focus_eval_f64": ([c_vp, c_vp, c_i64, c_i64, c_int, c_int] + [c_vp] * 7, c_int),
        "akb_sep_search_f64": ([c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_dbl, c_dbl, c_int, c_int,
                                c_dbl, c_dbl, c_vp, c_vp], c_int),
        "akb_chain_tilt_f64": ([ctypes.POINTER(ChainDesc), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64]
                               + [c_vp] * 6 + [ctypes.POINTER(LeafSink), c_vp], c_int),
        "akb_chain_tilt_opd_f64": ([ctypes.POINTER(ChainDesc), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                    c_vp, c_vp, ctypes.POINTER(LeafSink)] + [c_vp] * 8, c_int),
        "akb_opd_f64": ([c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp],
                        c_int),
        "akb_resample_f64": ([c_vp, c_vp, c_i64, c_vp], c_int),
        "akb_calc_ds_f64": ([c_vp, c_i64, c_int, c_int, c_vp, c_vp], c_int),
        "akb_plane_sweep_rows_f64": ([c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_int, c_vp, c_vp, c_vp], c_int),
        "akb_plane_sweep_sink_f64": ([c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_int, c_vp,
                                      ctypes.POINTER(LeafSink), c_vp], c_int),
        "akb_pupil_sample_f64": ([c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_leaf_sink_bytes": ([c_int, c_i64], c_i64),
        "akb_leaf_sink_layout": ([c_vp, c_int, c_int, c_i64, ctypes.POINTER(LeafSink)], c_int),
        "akb_leaf_finish_work_bytes": ([c_int, c_i64], c_i64),
        "akb_leaf_finish_f64": ([ctypes.POINTER(LeafSink), c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_leaf_parts_f64": ([ctypes.POINTER(LeafSink), c_vp, c_vp, c_int, c_vp, c_vp, c_vp], c_int),
        "akb_parts_chain_f64": ([c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "akb_pairwise_work_bytes": ([c_int, c_i64], c_i64),
        "akb_pairwise_sum_f64": ([c_vp, c_i64, c_int, c_i64, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_huygens_splits": ([c_i64, c_i64], c_int),
        "akb_huygens_work_bytes": ([c_i64, c_i64, c_int], c_i64),
        "akb_huygens_f64": ([c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_int, c_vp,
                             c_vp], c_int),
        "akb_scale_field_f64": ([c_vp, c_vp, c_i64, c_vp, c_vp], c_int),
        "akb_psf_work_bytes": ([c_int, c_int, c_int, c_int], c_i64),
        "akb_psf_f64": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_dbl, c_dbl, c_vp, c_vp, c_dbl, c_vp,
                         c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_psf_release_plans": ([], None),
        "akb_release_all": ([], None),
        "akb_selftest_arith_f64": ([c_vp, c_vp, c_i64, c_vp, c_vp], c_int),
        "akb_first_valid_rows_f64": ([c_vp, c_int, c_int, c_vp, c_vp], c_int),
        "akb_rotate_work_bytes": ([c_int, c_int], c_i64),
        "akb_rotate_with_nan_f64": ([c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_pupil_post_f64": ([c_vp, c_int, c_int, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_pupil_post_work_bytes": ([c_int, c_int], c_i64),
        "akb_moments_work_bytes": ([], c_i64),
        "akb_map_moments_f64": ([c_vp, c_int, c_int, c_int, c_vp, c_dbl, c_int, c_dbl, c_vp, c_vp, c_vp], c_int),
        "akb_plane_subtract_f64": ([c_vp, c_int, c_int, c_vp, c_vp, c_vp], c_int),
        "akb_legendre_rows_f64": ([c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
                                  c_int),
        "akb_gd_cells_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_dbl, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_gd_pockets": ([c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_valid_mask_u8": ([c_vp, c_int, c_int, c_vp, c_vp], c_int),
        "akb_external_contours": ([c_vp, c_int, c_int, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp], c_int),
        "akb_approx_poly_dp": ([c_vp, c_i32, c_dbl, c_int, c_vp, c_vp], c_int),
        "akb_affine_from_points": ([c_vp, c_vp, c_vp], c_int),
        "akb_affine_invert": ([c_vp, c_vp], c_int),
        "akb_warp_affine_f64": ([c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp], c_int),
        "akb_gd_check_pockets": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_dbl, c_vp, c_vp],
                                 c_int),
        "akb_gd_grad_sweeps_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                    c_vp, c_vp, c_dbl, c_dbl, c_int, c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_gd_eval_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int,
                             c_vp, c_vp, c_int, c_vp, c_vp, c_vp], c_int),
        "akb_gd_cone_work_bytes": ([c_int, c_int, c_int, c_int, c_int], c_i64),
        "akb_gd_patch_timing": ([c_int], c_int),
        "akb_gd_patch_order": ([c_int, c_vp], c_int),
        "akb_gd_patch_times": ([c_vp, c_vp, c_int], c_int),
        "akb_gd_band_times": ([c_vp, c_int], c_int),
        "akb_gd_patch_phases": ([c_vp], c_int),
        "akb_gd_axes_f64": ([c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_gd_claims_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                               c_int, c_vp, c_int, c_vp, c_vp, c_vp], c_int),
        "akb_gd_cone_part_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                  c_int, c_vp, c_int, c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp, c_vp], c_int),
        "akb_gd_part_finish_f64": ([c_vp, c_vp, c_i64, c_int, c_vp], c_int),
        "akb_gd_ring_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_gd_cells_window_f64": ([c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_dbl, c_vp, c_vp], c_int),
        "akb_gd_cone_eval_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                  c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_gd_cone_solve_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                   c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp], c_int),
        "akb_gd_cells_claims_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_dbl, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
                                     c_vp], c_int),
        "akb_gd_claim_pockets_f64": ([c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
                                      c_vp], c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res


def lib():
    """The loaded library. Raises (never falls back) when it is missing or cannot load."""
    global _LIB
    if _LIB is None:
        # AKB_LIB: another build of the same ABI (A/B timing of kernel variants); default the in-tree one
        path = os.environ.get("AKB_LIB") or _build.SO
        if not os.path.exists(path):
            raise AKBError(
                f"{path} is missing: build the HIP extension first (python -m akbraytracing_amd.build "
                "or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(path)
        _declare(L)
        if L.akb_abi_version() != ABI_VERSION:
            raise AKBError(f"{path} has ABI {L.akb_abi_version()}, the bindings expect {ABI_VERSION}: rebuild")
        if not os.environ.get("AKB_LIB") and os.path.isdir(_build.CSRC):
            # provenance: the library must be the build of this tree's sources (a prebuilt .so
            # shipped beside edited sources is refused, not silently run)
            want = _build.sources_hash()
            got = L.akb_sources_hash().decode()
            if got != want:
                raise AKBError(f"{path} was built from sources {got[:16]}, the tree's hash {want[:16]}: rebuild "
                               "(python -m akbraytracing_amd.build)")
        if L.akb_chain_desc_size() != ctypes.sizeof(ChainDesc):
            raise AKBError("akb_chain_desc layout mismatch between include/akb_raytrace.h and _lib.py")
        _LIB = L
        # the library's cached plans, device tables, pinned buffers and events are freed while the
        # HIP runtime is still up: Python's exit hooks run before the C runtime's static destructors
        # (left to those, rocFFT's teardown can run after HIP's)
        atexit.register(_release_all, L)
    return _LIB


def _release_all(L):
    try:
        L.akb_release_all()
    except Exception:  # exit path: never mask the process's own status
        pass


def sources_hash():
    """the akb_sources_hash() of the loaded library"""
    return lib().akb_sources_hash().decode()


def check(status):
    if status != 0:
        msg = lib().akb_last_error()
        raise AKBError(f"libakb_hip error {status}: {msg.decode() if msg else ''}")
