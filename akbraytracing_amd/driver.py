"""plot_result_debug(params, 'ray_wave', option_legendre=True) end to end on the device.

The reference's 'ray_wave' mode (AKB_raytrace_20250312.py:1326; trace :2694-2905, tilt
:3565-3601, OPD :3611-3690, post :3692-3775) is what its alignment loops call for every candidate
system (auto_focus_NA's tail, :12880-12884; the Legendre alignment scripts): build the system from
params, trace it in two passes, tilt, form DistError2 / Wave2, grid them with griddata(cubic),
plane-correct, compute the PSF, rectify the pupil map and fit Legendre terms, returning
(inner_products, orders, pvs). With install() alone the reference runs that mode itself and every
primitive call is a host <-> device round trip of (3, N) arrays; here the whole chain stays on the
device:

  geometry.build_akb        params -> quadrics, detector planes, launch grid (row a9)
  wavefront.RayWave.run     picks, pass 1, resample, pass 2, tilt, DistError2 / Wave2 (rows a1-a8)
  pupilmap.wave_maps        griddata(cubic) of DistError2 and Wave2 (one triangulation),
                            - nanmean, plane correction with the 3-sigma filter (row f1)
  psfcalc.psf_calc          rotation estimate, rotate_with_nan, pad-16 PSF, trim, .npy files (a13)
  affine.extract_affine_square_region, pupilmap.match_legendre_multi  (row f4)

The files the mode writes are written the same way (matrixWave2(nm).txt in the working directory -
and its .tiff when tifffile is importable -, the psf .npy files, matrixWave2_Corrected(lambda).txt,
rectified_img.txt, inner_products.csv, orders.csv under directory_name); its figures and console
diagnostics are not drawn / printed (plotting is out of scope), except the PV line. Parity: each
stage is pinned on its own (tests/test_gpu_parity.py, test_affine.py, test_oracle_golden.py); the
chain is checked against the oracle's composition of the same stages (tests/test_driver.py). cv2 is
absent from this image, so the reference's own run cannot reach its return value here: the
end-to-end answer's parity with the reference is unpinned past extract_affine_square_region.
"""
import os

import numpy as np

ASSES_ORDER = 5  # assesorder, :3743


def ray_wave_conditions(option_HighNA=True):
    """defocusWave (m) and lambda_ (nm) of the 'ray_wave' mode (:3612-3617)."""
    return (1e-2, 13.5) if option_HighNA else (1e-3, 1.35)


def plot_result_ray_wave(params, ray_num, *, source_shift=(0.0, 0.0, 0.0), option_set=True, option_HighNA=True,
                         option_energy="EUV", option_AKB=True, directory=None, workdir=None, verbose=True,
                         as_dict=False, option_legendre=True):
    """The 'ray_wave' mode with option_save=True for the AKB system built from params on a
    ray_num x ray_num grid. With option_legendre (the alignment loops' call) returns
    (inner_products, orders, pvs) as the reference (:3775); without it (the plotting run) writes the
    run's conditions file optical_params.txt (:3803-3834) and returns np.nanstd(map / lambda) * 6
    (:3913) - its figures are not drawn. np.inf where the reference returns np.inf (an unbuildable
    system). directory: the module's directory_name (psf_calc's and the txt / csv outputs);
    workdir: where the reference's cwd-relative 'matrixWave2(nm).txt' goes (default: the current
    directory). as_dict: also return the intermediate maps (device tensors)."""
    from . import geometry as G
    from .affine import extract_affine_square_region
    from .psfcalc import psf_calc
    from .pupilmap import match_legendre_multi, wave_maps
    from .wavefront import RayWave, SystemGeometry
    b = G.build_akb(params, source_shift=source_shift, option_set=option_set)
    if not isinstance(b, dict):
        return b
    defocus_wave, lambda_ = ray_wave_conditions(option_HighNA)
    det2 = np.zeros(10)
    det2[6] = 1
    det2[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]) + defocus_wave)  # coeffs_det2, :3618-3620
    b = dict(b, det2=[float(x) for x in det2], defocus_wave_m=defocus_wave)
    n = int(ray_num)
    run = RayWave(SystemGeometry.from_dict(b), n).run()
    m = wave_maps(run["detcenter2"], run["dist_err2"], run["wave2"], n, n)
    matrixWave2 = m["matrixWave2"].cpu().numpy()
    workdir = os.getcwd() if workdir is None else workdir
    np.savetxt(os.path.join(workdir, "matrixWave2(nm).txt"), matrixWave2)
    try:
        import tifffile
    except ImportError:
        tifffile = None
    if tifffile is not None and hasattr(tifffile, "imwrite"):
        tifffile.imwrite(os.path.join(workdir, "matrixWave2(nm).tiff"), matrixWave2)
    corrected = m["matrixWave2_Corrected"]
    corr = corrected.cpu().numpy()
    if verbose:
        print('PV', np.nanmax(corr) - np.nanmin(corr))
    grid_H = m["grid_H"] - np.mean(m["grid_H"])  # :3704-3705
    grid_V = m["grid_V"] - np.mean(m["grid_V"])
    psf = psf_calc(corrected, grid_H, grid_V, defocus_wave, option_energy=option_energy, option_AKB=option_AKB,
                   directory=directory)
    out_dir = directory if directory is not None else "."
    os.makedirs(out_dir, exist_ok=True)
    wave_lambda = corr / lambda_
    np.savetxt(os.path.join(out_dir, 'matrixWave2_Corrected(lambda).txt'), wave_lambda)
    rectified_img = extract_affine_square_region(wave_lambda, target_size=matrixWave2.shape[0])
    np.savetxt(os.path.join(out_dir, 'rectified_img.txt'), rectified_img)
    fit_datas, inner_products, orders = match_legendre_multi(rectified_img[1:-2, 1:-2], ASSES_ORDER)
    length = len(inner_products)
    pvs = np.zeros(length + 1)
    for i in range(length):
        pvs[i] = (np.nanmax(fit_datas[i]) - np.nanmin(fit_datas[i])) * np.sign(inner_products[i])
    np.savetxt(os.path.join(out_dir, 'inner_products.csv'), inner_products, delimiter=',')
    np.savetxt(os.path.join(out_dir, 'orders.csv'), orders, delimiter=',')
    pv6 = np.nanstd(wave_lambda) * 6
    if option_legendre:
        pvs[-1] = pv6 * np.sign(np.sum(inner_products))
    else:  # the plotting run: its conditions file (:3803-3834), then it returns the 6-sigma (:3913)
        p = np.asarray(params, dtype=np.float64).ravel()
        with open(os.path.join(out_dir, 'optical_params.txt'), 'w') as f:
            f.write("input\n")
            f.write("====================\n")
            for i in range(26):
                f.write(f"params[{i}]: {p[i]}\n")
    if as_dict:
        return dict(inner_products=inner_products, orders=orders, pvs=pvs, maps=m, run=run, psf=psf,
                    rectified_img=rectified_img, fit_datas=fit_datas, grid_H=grid_H, grid_V=grid_V, pv=pv6)
    if option_legendre:
        return inner_products, orders, pvs
    return pv6



def kb_ray_wave_conditions(option_HighNA=True, option_energy="EUV", widesearch=False):
    """defocusWave (m) and lambda_ (nm) of KB_debug's 'ray_wave' mode (:11726-11739)."""
    if not option_HighNA:
        return 1e-5, 1.35
    lam = {"EUV": 13.5, "hardXray": 0.135, "softXray": 1.35}.get(option_energy)
    if lam is None:
        raise ValueError(f"option_energy {option_energy!r}: the reference leaves lambda_ unset")
    return (1e-1 if widesearch else 1e-4), lam


KB_RECTIFIED_SIZE = 256  # extract_affine_square_region(..., target_size=256), :11827


def kb_ray_wave(params, ray_num, *, source_shift=(0.0, 0.0, 0.0), designparams=None, option_HighNA=True,
                option_energy="EUV", widesearch=False, option_legendre=True, directory=None, workdir=None,
                verbose=True, as_dict=False):
    """KB_debug(params, na_ratio_h, na_ratio_v, 'ray_wave', option_legendre, source_shift,
    option_save=True) (:11725-11879) for the KB pair of geometry.build_kb on a ray_num x ray_num
    grid: one trace (the mode takes no equal-angle resample, :11001), the np.mean tilt
    (:11703-11717), DistError2 / Sph / Wave2 (:11740-11779), griddata(cubic) of Wave2 and the plane
    correction, psf_calc (option_AKB False), the pupil map rectified to 256 x 256 and its Legendre
    fit. Writes the mode's files (matrixWave2(nm).txt in workdir; matrixWave2_Corrected(lambda).txt,
    rectified_img.txt, inner_products.txt, orders.txt, pvs.txt, fit_sum.txt, pv.txt and psf_calc's
    .npy files under directory). Returns (inner_products, orders, pvs) with option_legendre, else
    pv (6 sigma of the map in waves) after writing optical_params.txt as the plotting run does (its
    figures are not drawn); np.inf for an unbuildable system.

    The device trace is RayWave's with resample_pass=False, whose nanmeans are np.mean's bits when
    no ray misses; a ray that misses makes the reference's np.mean NaN everywhere, and raises here."""
    from . import _lib
    from . import geometry as G
    from .affine import extract_affine_square_region
    from .psfcalc import psf_calc
    from .pupilmap import match_legendre_multi, wave_maps
    from .wavefront import RayWave, SystemGeometry
    import torch
    b = G.build_kb(params, source_shift=source_shift, designparams=designparams)
    if not isinstance(b, dict):
        return b
    defocus_wave, lambda_ = kb_ray_wave_conditions(option_HighNA, option_energy, widesearch)
    det2 = np.zeros(10)
    det2[6] = 1
    det2[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]) + defocus_wave)  # coeffs_det2, :11740-11742
    b = dict(b, det2=[float(x) for x in det2], defocus_wave_m=defocus_wave)
    n = int(ray_num)
    run = RayWave(SystemGeometry.from_dict(b), n, resample_pass=False).run()
    if bool(torch.isnan(run["wave2"]).any()):
        raise _lib.AKBError("KB 'ray_wave': a ray missed a mirror or the detector; the reference's np.mean "
                            "makes every value NaN there")
    m = wave_maps(run["detcenter2"], run["dist_err2"], run["wave2"], n, n)
    matrixWave2 = m["matrixWave2"].cpu().numpy()
    workdir = os.getcwd() if workdir is None else workdir
    np.savetxt(os.path.join(workdir, "matrixWave2(nm).txt"), matrixWave2)
    try:
        import tifffile
    except ImportError:
        tifffile = None
    if tifffile is not None and hasattr(tifffile, "imwrite"):
        tifffile.imwrite(os.path.join(workdir, "matrixWave2(nm).tiff"), matrixWave2)
    corrected = m["matrixWave2_Corrected"]
    corr = corrected.cpu().numpy()
    grid_H = m["grid_H"] - np.mean(m["grid_H"])  # :11799-11800
    grid_V = m["grid_V"] - np.mean(m["grid_V"])
    psf = psf_calc(corrected, grid_H, grid_V, defocus_wave, option_energy=option_energy, option_AKB=False,
                   directory=directory)
    if verbose:
        print('PV', np.nanmax(corr) - np.nanmin(corr))
    out_dir = directory if directory is not None else "."
    os.makedirs(out_dir, exist_ok=True)
    wave_lambda = corr / lambda_
    np.savetxt(os.path.join(out_dir, 'matrixWave2_Corrected(lambda).txt'), wave_lambda)
    pv = np.nanstd(wave_lambda) * 6
    rectified_img = extract_affine_square_region(wave_lambda, target_size=KB_RECTIFIED_SIZE)
    np.savetxt(os.path.join(out_dir, 'rectified_img.txt'), rectified_img)
    fit_datas, inner_products, orders = match_legendre_multi(rectified_img[1:-2, 1:-2], ASSES_ORDER)
    length = len(inner_products)
    pvs = np.zeros(length + 1)
    for i in range(length):
        pvs[i] = (np.nanmax(fit_datas[i]) - np.nanmin(fit_datas[i])) * np.sign(inner_products[i])
    fit_sum = np.sum(fit_datas, axis=0)
    np.savetxt(os.path.join(out_dir, 'inner_products.txt'), inner_products)
    np.savetxt(os.path.join(out_dir, 'orders.txt'), orders)
    np.savetxt(os.path.join(out_dir, 'pvs.txt'), pvs)
    np.savetxt(os.path.join(out_dir, 'fit_sum.txt'), fit_sum)
    np.savetxt(os.path.join(out_dir, 'pv.txt'), np.array([pv]))
    if option_legendre:
        pvs[-1] = np.nanstd(wave_lambda) * 6 * np.sign(np.sum(inner_products))
    else:  # the plotting run's conditions file (:11907-11938); it returns pv (:11942)
        p = np.asarray(params, dtype=np.float64).ravel()
        with open(os.path.join(out_dir, 'optical_params.txt'), 'w') as f:
            f.write("input\n")
            f.write("====================\n")
            for i in range(26):
                f.write(f"params[{i}]: {p[i]}\n")
    if as_dict:
        return dict(inner_products=inner_products, orders=orders, pvs=pvs, maps=m, run=run, psf=psf,
                    rectified_img=rectified_img, fit_datas=fit_datas, fit_sum=fit_sum, grid_H=grid_H, grid_V=grid_V,
                    pv=pv)
    if option_legendre:
        return inner_products, orders, pvs
    return pv
