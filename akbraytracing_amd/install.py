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

The driver's steps after the trace are rebound too: griddata (the module's
`from scipy.interpolate import griddata`, :28), plane_correction_with_nan_and_outlier_filter,
psf_calc (reading the module's live option_energy / option_AKB / directory_name as the reference
does, :1161-1166, :1202-1214, :1271-1273), find_defocus and calc_dS. plot_result_debug's 'test'
mode and auto_focus_NA (:12746) run the batched device search (autofocus.py) for the live Wolter
III+I AKB system, its 'sep' mode and compare_sep (:9267) the one-launch plane searches (sep.py),
and its 'ray_wave' mode with option_legendre (the alignment loops' call) the whole chain from
params to the Legendre fit (driver.py); the reference's auto_focus_sep, calc_FoC and alignment
loops reach them through the module globals.
install(mod, names=[...]) picks a subset; uninstall(mod) restores every original.

The wrappers read the module's live `option_mpmath` flag (AKB_raytrace_20250312.py:92) at call
time and hand the call to the original function when it is set (the mpmath branch, :399-443).
"""
from . import primitives as _P
from . import psf as _psf
from . import wavecalc as _W


def _lazy(modname, attr):
    def call(*args, **kwargs):
        import importlib
        return getattr(importlib.import_module(f"{__package__}.{modname}"), attr)(*args, **kwargs)
    return call


def _psf_calc_for(mod):
    """psf_calc with the module's globals, as the reference's psf_calc reads them."""
    def psf_calc(matrixWave2_Corrected, grid_H, grid_V, defocusWave):
        from .psfcalc import psf_calc as native
        native(matrixWave2_Corrected, grid_H, grid_V, defocusWave,
               option_energy=getattr(mod, "option_energy", "EUV"), option_AKB=getattr(mod, "option_AKB", True),
               directory=getattr(mod, "directory_name", None))
        return None  # the reference's psf_calc returns nothing; its results are the .npy files
    return psf_calc

def _akb_native_ok(mod):
    """The batched focus search restates the Wolter III+I system of the live plot_result_debug
    (:1325 `if option_wolter_3_1`) for option_AKB; anything else stays the reference's."""
    return (getattr(mod, "option_AKB", False) and getattr(mod, "option_wolter_3_1", False)
            and not getattr(mod, "option_mpmath", False))


def _kb_native_ok(mod):
    """KB_debug's pair as build_kb restates it: option_AKB False, the KB_define design branch
    (optKBdesign False, :65, :9748) with option_HighNA (:83, :9938) and both mirrors traced
    (option_2mirror, :66)."""
    return (not getattr(mod, "option_AKB", True) and not getattr(mod, "optKBdesign", False)
            and getattr(mod, "option_HighNA", True) and getattr(mod, "option_2mirror", True)
            and not getattr(mod, "option_mpmath", False))


def _kb_debug_for(mod, original):
    """KB_debug (:9742) with its 'test' mode (auto_focus_NA's, called hundreds of times for a KB
    system; autofocus.kb_test), its 'sep' mode (auto_focus_sep's; sep.kb_sep), its 'wave' mode
    (saveWaveData's; wavedata.kb_wave) and its 'ray_wave' mode (driver.kb_ray_wave) on the device,
    with the
    module's live KBdesign_7params (:100); every other mode runs the reference's own function."""
    def KB_debug(params, na_ratio_h, na_ratio_v, option, option_legendre=False, source_shift=[0., 0., 0.],
                 option_save=True, designparams=None):
        dp = designparams if designparams is not None else getattr(mod, "KBdesign_7params", None)
        if option == "test" and _kb_native_ok(mod):
            from .autofocus import kb_test
            return kb_test(params, source_shift, designparams=dp)
        if (option == "wave" and _kb_native_ok(mod) and getattr(mod, "option_rotate", True)
                and not getattr(mod, "option_avrgsplt", False)
                and getattr(mod, "wave_num_H", 0) == getattr(mod, "wave_num_V", 1)):
            from .wavedata import kb_wave
            return kb_wave(params, mod.wave_num_H, defocus_for_wave=getattr(mod, "defocusForWave", 1e-3),
                           source_shift=source_shift, designparams=dp)
        if option == "sep" and _kb_native_ok(mod):
            from .sep import kb_sep
            return kb_sep(params, source_shift, designparams=dp, widesearch=bool(getattr(mod, "widesearch", False)))
        if (option == "ray_wave" and option_save and _kb_native_ok(mod)
                and getattr(mod, "wave_num_H", 0) == getattr(mod, "wave_num_V", 1)):
            # the whole mode on the device (driver.kb_ray_wave), its figures not drawn
            from .driver import kb_ray_wave
            return kb_ray_wave(params, mod.wave_num_H, source_shift=source_shift, designparams=dp,
                               option_HighNA=getattr(mod, "option_HighNA", True),
                               option_energy=getattr(mod, "option_energy", "EUV"),
                               widesearch=bool(getattr(mod, "widesearch", False)), option_legendre=option_legendre,
                               directory=getattr(mod, "directory_name", None))
        return original(params, na_ratio_h, na_ratio_v, option, option_legendre=option_legendre,
                        source_shift=source_shift, option_save=option_save, designparams=designparams)
    return KB_debug


def _plot_result_debug_for(mod, original):
    """plot_result_debug with its 'test' mode (the one auto_focus_NA and the alignment loops call
    hundreds of times), its 'sep' mode (auto_focus_sep's, sep.py), its 'wave' mode and its 'ray_wave'
    mode (driver.py: with option_legendre the alignment loops' call, without it the plotting run -
    the same device chain and files, its figures not drawn) on the device; every other mode runs the
    reference's own function, whose primitives install() has rebound."""
    def plot_result_debug(params, option, source_shift=[0., 0., 0.], option_tilt=True, option_legendre=False,
                          angular_shift=[0., 0.], option_save=True):
        if option == "test" and _akb_native_ok(mod) and list(angular_shift) == [0., 0.]:
            from .autofocus import plot_result_test
            return plot_result_test(params, source_shift, option_tilt, option_set=bool(getattr(mod, "option_set", False)))
        if option == "sep" and _akb_native_ok(mod) and list(angular_shift) == [0., 0.]:
            from .sep import plot_result_sep
            return plot_result_sep(params, source_shift, option_tilt, option_set=bool(getattr(mod, "option_set", False)),
                                   widesearch=bool(getattr(mod, "widesearch", False)))
        if (option == "ray_wave" and option_save and option_tilt and _akb_native_ok(mod)
                and list(angular_shift) == [0., 0.] and getattr(mod, "wave_num_H", 0) == getattr(mod, "wave_num_V", 1)):
            # the whole chain on the device (driver.py): the alignment loops' call (option_legendre)
            # and the live __main__ plotting run (:14603-14611; its figures not drawn)
            from .driver import plot_result_ray_wave
            return plot_result_ray_wave(params, mod.wave_num_H, source_shift=source_shift,
                                        option_set=bool(getattr(mod, "option_set", False)),
                                        option_HighNA=getattr(mod, "option_HighNA", True),
                                        option_energy=getattr(mod, "option_energy", "EUV"), option_AKB=True,
                                        directory=getattr(mod, "directory_name", None),
                                        option_legendre=bool(option_legendre))
        if (option == "wave" and _akb_native_ok(mod) and list(angular_shift) == [0., 0.]
                and getattr(mod, "option_rotate", True) and getattr(mod, "wave_num_H", 0) == getattr(mod, "wave_num_V", 1)):
            from .wavedata import plot_result_wave
            return plot_result_wave(params, mod.wave_num_H, defocus_for_wave=getattr(mod, "defocusForWave", 1e-3),
                                    option_set=bool(getattr(mod, "option_set", False)), source_shift=source_shift)
        return original(params, option, source_shift=source_shift, option_tilt=option_tilt,
                        option_legendre=option_legendre, angular_shift=angular_shift, option_save=option_save)
    return plot_result_debug


def _auto_focus_for(mod, original):
    """auto_focus_NA (:12746) with every sweep on the device, reading the module's live flags
    (widesearch :98, option_set :94, option_AKB :80) as the reference does: the Wolter III+I
    system's sweeps or KB_debug's pair's; the mpmath branch and other systems run the reference's
    own function."""
    def auto_focus_NA(num_adj_astg, initial_params, na_ratio_h, na_ratio_v, option, option_param,
                      option_disp='ray', option_mode=False, source_shift0=[0., 0., 0.], option_legendre=False):
        kb = _kb_native_ok(mod)
        if not (_akb_native_ok(mod) or kb):
            return original(num_adj_astg, initial_params, na_ratio_h, na_ratio_v, option, option_param,
                            option_disp=option_disp, option_mode=option_mode, source_shift0=source_shift0,
                            option_legendre=option_legendre)
        from .autofocus import auto_focus_NA as native
        return native(num_adj_astg, initial_params, na_ratio_h, na_ratio_v, option, option_param,
                      option_disp=option_disp, option_mode=option_mode, source_shift0=source_shift0,
                      option_legendre=option_legendre, widesearch=bool(getattr(mod, "widesearch", False)),
                      option_set=bool(getattr(mod, "option_set", False)), option_AKB=not kb,
                      kb_design=getattr(mod, "KBdesign_7params", None), driver=mod)
    return auto_focus_NA


def _compare_sep_for(mod, original):
    """compare_sep (:9267) with its twenty plane searches in one device launch (sep.py), reading the
    module's live widesearch flag (:98) as the reference does."""
    def compare_sep(rays, points, coeffs_det0, ray_num, region):
        from .sep import compare_sep as native
        return native(rays, points, coeffs_det0, ray_num, region, widesearch=bool(getattr(mod, "widesearch", False)))
    return compare_sep


def _save_wave_for(mod, original):
    """saveWaveData (:13475) with the 'wave' trace, calc_dS and the grids on the device, reading
    the module's flags (wave_num_H / V, defocusForWave, downsample_*, option_HighNA, option_2mirror,
    option_avrgsplt, option_set) as the reference does, and ending the process with sys.exit() as
    it does (:13763); KB_debug's pair (option_AKB False) through wavedata.kb_wave."""
    def saveWaveData(initial_params, ysize=1e-6, zsize=1e-6):
        kb = _kb_native_ok(mod) and not getattr(mod, "option_avrgsplt", False)
        if not ((_akb_native_ok(mod) or kb) and getattr(mod, "option_rotate", True)):
            return original(initial_params, ysize=ysize, zsize=zsize)
        import sys
        from .wavedata import saveWaveData as native
        g = lambda k, d: getattr(mod, k, d)  # noqa: E731
        native(initial_params, ysize, zsize, ray_num_H=g("wave_num_H", 65), ray_num_V=g("wave_num_V", 65),
               defocus_for_wave=g("defocusForWave", 1e-3),
               downsample=tuple(g(k, 0) for k in ("downsample_h1", "downsample_v1", "downsample_h2", "downsample_v2",
                                                  "downsample_h_f", "downsample_v_f")),
               option_set=bool(g("option_set", False)), option_HighNA=g("option_HighNA", True),
               option_2mirror=g("option_2mirror", True), option_avrgsplt=g("option_avrgsplt", False),
               option_AKB=not kb, kb_design=g("KBdesign_7params", None))
        sys.exit()
    return saveWaveData


_PER_MODULE = {"plot_result_debug": _plot_result_debug_for, "auto_focus_NA": _auto_focus_for, "KB_debug": _kb_debug_for,
               "saveWaveData": _save_wave_for, "compare_sep": _compare_sep_for}

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
    "griddata": _lazy("griddata", "griddata"),
    "plane_correction_with_nan_and_outlier_filter": _lazy("pupilmap", "plane_correction_with_nan_and_outlier_filter"),
    "find_defocus": _lazy("focus", "find_defocus"),
    "calc_dS": _lazy("wavedata", "calc_dS"),
    "extract_affine_square_region": _lazy("affine", "extract_affine_square_region"),
    "psf_calc": None,  # bound per module (_psf_calc_for)
    "plot_result_debug": None,  # bound per module (_PER_MODULE)
    "KB_debug": None,
    "auto_focus_NA": None,
    "saveWaveData": None,
    "compare_sep": None,
}
# every name install() can rebind (pass a subset as `names`)
NATIVE_NAMES = tuple(_NATIVE)
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
    """Rebind `names` (default: every hot-path name the module defines, NATIVE_NAMES) in `mod`.
    Returns the list of rebound names. uninstall(mod) restores the originals.

    Parity unpinned: extract_affine_square_region (AKB_raytrace_20250312.py:1047-1119) restates
    OpenCV's findContours / approxPolyDP / warpAffine; cv2 is not importable here and the reference
    holds no recorded output of it, so it is checked only against oracle/affine.py and closed forms.
    Leave it out of `names` to keep the reference's cv2 step."""
    done = []
    for name in (names or _NATIVE):
        if name not in _NATIVE or not hasattr(mod, name):
            continue
        cur = getattr(mod, name)
        if getattr(cur, "__akb_native__", False):
            done.append(name)
            continue
        if name in _PER_MODULE:
            w = _PER_MODULE[name](mod, cur)
            w.__wrapped__ = cur
            w.__akb_native__ = True
            setattr(mod, name, w)
            done.append(name)
            continue
        native = _NATIVE[name] if _NATIVE[name] is not None else _psf_calc_for(mod)
        setattr(mod, name, _wrap(mod, name, cur, native))
        done.append(name)
    return done


def uninstall(mod):
    for name in _NATIVE:
        cur = getattr(mod, name, None)
        if cur is not None and getattr(cur, "__akb_native__", False):
            setattr(mod, name, cur.__wrapped__)
