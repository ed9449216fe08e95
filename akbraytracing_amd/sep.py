"""plot_result_debug's 'sep' analysis and auto_focus_sep on the device.

plot_result_debug(params, 'sep') (AKB_raytrace_20250312.py:1326) traces its 53 x 53 grid in two
passes with the equal-angle resample (:2849-2905), tilts the exit rays by their nanmean angles
about the mean detector hit (:3565-3601) and hands them to compare_sep (:9267-9560): twenty
coarse-to-fine searches (optimize_min_index, :9174-9217) for the plane x = -a that minimises
sqrt(np.std(z)^2 + np.std(y)^2) of a ray subset - the three grid rows and columns (r / y / g),
their first two thirds and last third, and two diagonals - then the mean hit positions of those
rows and columns on the last searched plane. auto_focus_sep (:12897-13318) runs auto_focus_NA +
'sep' for five values of one alignment parameter and forms the aberration measures from them.

Here:
  two_pass_trace   the shared two-pass device trace (wavedata.two_pass_trace)
  the tilt         theta from np.nanmean(np.arctan(...)) on the host (numpy's SIMD arctan has no
                   bitwise device equivalent; one 53^2 array), rotations and the focus mean on the
                   device in the reference's dgemm / pairwise order (primitives, reduce)
  compare_sep      akb_sep_search_f64: all twenty searches in ONE launch, one workgroup per search
                   and one lane per linspace point, the whole shrink loop inside the kernel, every
                   np.std in numpy's pairwise order (the reference evaluates ~26000 numpy plane
                   intersections, one Python call each)
  auto_focus_sep   the reference's loop over the native auto_focus_NA (autofocus.py) and 'sep'.
so the twelve outputs and the abrr / matrix answers are the reference's bit for bit
(tests/golden/akb_sep.npz). The reference's 'matrix' figures are not drawn (plotting is out of
scope); its linear fits are scikit-learn's, as the reference's.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from . import device as D
from . import primitives as P

SEP_OUTPUTS = ("focus_v0", "focus_h0", "pos_v0", "pos_h0", "std_v0", "std_h0", "focus_v0_l", "focus_h0_l",
               "focus_v0_u", "focus_h0_u", "focus_std_obl1", "focus_std_obl2")


def sep_subsets(ray_num, n_rays):
    """compare_sep's twenty index sets as (start, step, count), in its call order (:9278-9304:
    thinned_array_h_r/y/g are grid rows, _v_r/y/g grid columns; :9334-9541: whole, [:2/3], [:-2/3]
    of each, then the two diagonals)."""
    n = int(ray_num)
    if n < 2:
        raise ValueError("compare_sep needs ray_num >= 2 (its diagonal step is ray_num - 1)")
    NN = n * n

    def rng_len(start, stop, step):
        return len(range(start, stop, step))

    a, b = round(n * (n - 1) / 2), round(n * (n + 1) / 2)
    sy = round((n - 1) / 2)
    rows = [(0, 1, len(range(n + 1)[0:n])), (a, 1, len(range(b + 1)[a:b])), (NN - n, 1, len(range(NN + 1)[NN - n:NN]))]
    cols = [(0, n, rng_len(0, NN, n)), (sy, n, rng_len(sy, NN, n)), (n - 1, n, rng_len(n - 1, NN, n))]
    whole = rows + cols
    lower = [(s, st, c * 2 // 3) for s, st, c in whole]
    upper = [(s, st, (c - c * 2 // 3) if c * 2 // 3 > 0 else 0) for s, st, c in whole]  # x[:-0] is empty
    obl1 = (n - 1, n - 1, max(rng_len(n - 1, n_rays, n - 1) - 1, 0))
    obl2 = (0, n + 1, rng_len(0, n_rays, n + 1))
    return whole + lower + upper + [obl1, obl2]


def compare_sep(rays, points, coeffs_det0, ray_num, region=1e-4, *, widesearch=False, verbose=True):
    """compare_sep (:9267-9560) with the reference's signature and returns. coeffs_det0 is updated in
    place as the reference's is (its searches write coeffs_det0[6] = 1 and coeffs_det0[9] = the
    plane being evaluated, so the last searched plane stays there and gives pos_v0 / pos_h0).
    widesearch: the module flag (:98), +-0.1 instead of +-0.01 around coeffs_det0[9]. `region` is
    unused, as in the reference."""
    L = _lib.lib()
    R = D.to_dev(rays)
    Q = D.to_dev(points)
    if R.dim() != 2 or R.shape[0] != 3 or tuple(Q.shape) != tuple(R.shape):
        raise ValueError("rays and points must both be (3, N)")
    N = int(R.shape[1])
    sub = sep_subsets(ray_num, N)
    S = len(sub)
    starts = (ctypes.c_int64 * S)(*[s for s, _, _ in sub])
    steps = (ctypes.c_int64 * S)(*[st for _, st, _ in sub])
    counts = (ctypes.c_int64 * S)(*[c for _, _, c in sub])
    for s, st, c in sub:
        if c > 0 and not (0 <= s < N and 0 <= s + (c - 1) * st < N):
            raise IndexError(f"index {s + (c - 1) * st} is out of bounds for axis 1 with size {N}")
    w = 1e-1 if widesearch else 1e-2
    c9 = np.float64(coeffs_det0[9])
    x_min, x_max = c9 - w, c9 + w
    out = torch.empty((S, 4), dtype=D.F64, device=R.device)
    _lib.check(L.akb_sep_search_f64(D.ptr(R), D.ptr(Q), N, N, S, starts, steps, counts, float(x_min), float(x_max),
                                    100, 20, 0.1, 1e-13, D.ptr(out), D.stream_handle()))
    o = out.cpu().numpy()
    if verbose:
        for q in range(S):
            if o[q, 3] > 1e-13:
                print('x_max - x_min', np.float64(o[q, 3]))
    coeffs_det0[6] = 1.
    coeffs_det0[9] = np.float64(o[S - 1, 2])
    foc = [np.float64(v) for v in o[:, 0]]
    std = [np.float64(v) for v in o[:, 1]]
    det = P.plane_ray_intersection(np.asarray(coeffs_det0, dtype=np.float64), R, Q).cpu().numpy()
    n = int(ray_num)
    d2r, d2y, d2g = det[:, ::n], det[:, round((n - 1) / 2)::n], det[:, n - 1::n]
    d1r = det[:, :n]
    d1y = det[:, round(n * (n - 1) / 2): round(n * (n + 1) / 2)]
    d1g = det[:, -n:]
    pos_v0 = np.array([[np.mean(d1r, axis=1)], [np.mean(d1y, axis=1)], [np.mean(d1g, axis=1)]])
    pos_h0 = np.array([[np.mean(d2r, axis=1)], [np.mean(d2y, axis=1)], [np.mean(d2g, axis=1)]])
    return (np.array(foc[0:3]), np.array(foc[3:6]), pos_v0, pos_h0, np.array(std[0:3]), np.array(std[3:6]),
            np.array(foc[6:9]), np.array(foc[9:12]), np.array(foc[12:15]), np.array(foc[15:18]), foc[18], foc[19])


def plot_result_sep(params, source_shift=(0.0, 0.0, 0.0), option_tilt=True, *, option_set=True, widesearch=False,
                    ray_num=53, verbose=True):
    """plot_result_debug(params, 'sep') (:1326; :2849-2905, :3565-3606) for the Wolter III+I AKB
    system built from params (geometry.build_akb): compare_sep's twelve outputs, or np.inf where the
    reference returns np.inf."""
    from . import geometry as G
    b = G.build_akb(params, source_shift=source_shift, option_set=option_set)
    if not isinstance(b, dict):
        return b
    if not option_tilt:
        # the reference reaches compare_sep with reflect4_rotated unbound (:3605)
        raise UnboundLocalError("local variable 'reflect4_rotated' referenced before assignment")
    return _sep_of_built(b, int(ray_num), np.nanmean, widesearch, verbose)


def kb_sep(params, source_shift=(0.0, 0.0, 0.0), *, designparams=None, widesearch=False, ray_num=53,
           verbose=True):
    """KB_debug(params, na_ratio_h, na_ratio_v, 'sep') (:9742; reset_p0's resample :11001-11054,
    the np.mean tilt :11703-11717, compare_sep :11719-11721) for the KB pair of geometry.build_kb:
    compare_sep's twelve outputs, or np.inf where the reference returns np.inf."""
    from . import geometry as G
    b = G.build_kb(params, source_shift=source_shift, designparams=designparams)
    if not isinstance(b, dict):
        return b
    return _sep_of_built(b, int(ray_num), np.mean, widesearch, verbose)


def _sep_of_built(b, n, mean, widesearch, verbose):
    """The two-pass trace, the tilt by mean(arctan) of the exit slopes (np.nanmean in
    plot_result_debug, np.mean in KB_debug), the rotation about np.mean(detcenter) and compare_sep
    on the plane x = s2f_middle + defocus."""
    from .reduce import means_to_host, np_sum
    from .wavedata import two_pass_trace
    hits, refl, det = two_pass_trace(b, n, "sep")
    ang = refl.cpu().numpy()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)  # nanmean of an all-NaN trace warns, gives NaN
        theta_y = -mean(np.arctan(ang[2, :] / ang[0, :]))
        theta_z = mean(np.arctan(ang[1, :] / ang[0, :]))
    refl_rot = P.rotate_vectors(refl, -theta_y, -theta_z)
    (focus,) = means_to_host([np_sum(det)])  # np.mean(detcenter, axis=1) (:3591, :11708)
    pts_rot = P.rotate_points(hits[-1], focus, -theta_y, -theta_z)
    coeffs_det = np.zeros(10)
    coeffs_det[6] = 1
    coeffs_det[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]))
    return compare_sep(refl_rot, pts_rot, coeffs_det, n, 1e-4, widesearch=widesearch, verbose=verbose)


def _abrr(sep):
    """The aberration measures of auto_focus_sep's 'abrr' branch (:12905-12948), one 'sep' result."""
    (focus_v0, focus_h0, _, _, _, _, focus_v0_l, focus_h0_l, focus_v0_u, focus_h0_u, focus_std_obl1,
     focus_std_obl2) = sep
    coma_v0 = focus_v0_l - focus_v0_u
    coma_h0 = focus_h0_l - focus_h0_u
    coma_v0_edge = (coma_v0[0] - np.mean(coma_v0) + coma_v0[2] - np.mean(coma_v0)) / 2.
    coma_h0_edge = (coma_h0[0] - np.mean(coma_h0) + coma_h0[2] - np.mean(coma_h0)) / 2.
    focus_len_v0 = focus_v0[0] - np.mean(focus_v0) - (focus_v0[2] - np.mean(focus_v0))
    coma_h_v0 = ((focus_v0_l[1] - focus_v0_u[1]) + (focus_v0_l[0] - focus_v0_u[0] + focus_v0_l[2] - focus_v0_u[2]) / 2) / 2
    oblique_ast = focus_std_obl1 - focus_std_obl2
    focus_len_h0 = focus_h0[0] - np.mean(focus_h0) - (focus_h0[2] - np.mean(focus_h0))
    coma_v_h0 = ((focus_h0_l[1] - focus_h0_u[1]) + (focus_h0_l[0] - focus_h0_u[0] + focus_h0_l[2] - focus_h0_u[2]) / 2) / 2
    coma_valance_v0 = coma_v0[0] - np.mean(coma_v0) - (coma_v0[2] - np.mean(coma_v0))
    coma_valance_h0 = coma_h0[0] - np.mean(coma_h0) - (coma_h0[2] - np.mean(coma_h0))
    coma_valance_cnt_edg_v0 = coma_v0[1] - np.mean(coma_v0) - coma_v0_edge
    coma_valance_cnt_edg_h0 = coma_h0[1] - np.mean(coma_h0) - coma_h0_edge
    return dict(a0=oblique_ast, a1=coma_v_h0, a2=coma_h_v0, a3=focus_len_h0, a4=focus_len_v0,
                a6=coma_valance_cnt_edg_h0, a7=coma_valance_cnt_edg_v0, a8=coma_valance_h0, a9=coma_valance_v0)


_ABRR_SETS = {"9": "a0 a1 a2 a3 a4 a6 a7 a8 a9", "7": "a0 a3 a4 a6 a7 a8 a9", "7coma": "a0 a1 a2 a3 a4 a8 a9",
              "5": "a0 a3 a4 a8 a9", "5coma": "a0 a1 a2 a3 a4", "2": "a1 a2", "3": "a0 a3 a4", "KB": "a0 a2 a4"}


def _linearfit(a, b, verbose):
    """auto_focus_sep's linearfit (:13121-13139): scikit-learn's LinearRegression and r2_score."""
    from sklearn.linear_model import LinearRegression
    from sklearn.metrics import r2_score
    model = LinearRegression()
    model.fit(a, b)
    slope = model.coef_[0]
    intercept = model.intercept_
    r2 = r2_score(b, model.predict(a))
    if r2 < 0.9:
        if verbose:
            print(f"R^2 score: {r2:.4f}")
            print("No correlation")
        return 0., np.mean(b), r2
    if verbose:
        print(f"Regression equation: b = {slope:.9f} * a + {intercept:.9f}")
        print(f"R^2 score: {r2:.4f}")
    return slope, intercept, r2


def auto_focus_sep(initial_params0, adj_param1, adj_param2, la, ua, option='none', option_eval=None, *,
                   widesearch=False, option_set=True, option_AKB=True, kb_design=None, verbose=True):
    """auto_focus_sep (:12897-13318): auto_focus_NA and the 'sep' analysis on the device for each of
    the five values of params[adj_param1] = params[adj_param2], the reference's measures, and its
    returns ('abrr': the measure vector of one 'sep' run of the focused params; 'matrix': the fitted
    slopes / intercepts per option_eval; otherwise None). option_AKB False: KB_debug's pair
    (auto_focus_NA's KB sweeps, kb_sep; the KB measure set a0, a2, a4 by default, :12978, :13158;
    kb_design: the module's KBdesign_7params). The reference's figures ('matrix') are not drawn."""
    from .autofocus import _SystemCache, auto_focus_NA
    cache = _SystemCache(option_set, 53, "akb" if option_AKB else "kb", kb_design)

    def focus(p):
        return auto_focus_NA(50, p, 1, 1, False, '', widesearch=widesearch, option_set=option_set,
                             option_AKB=option_AKB, kb_design=kb_design, verbose=verbose, cache=cache)

    def sep(p):
        if not option_AKB:
            return kb_sep(p, designparams=kb_design, widesearch=widesearch, verbose=verbose)
        return plot_result_sep(p, option_set=option_set, widesearch=widesearch, verbose=verbose)

    if option == 'abrr':
        _, _, initial_params = focus(initial_params0)
        m = _abrr(sep(initial_params))
        keys = _ABRR_SETS.get(option_eval, _ABRR_SETS["9" if option_AKB else "KB"]).split()
        return np.array([m[k] for k in keys])

    initial_params = initial_params0.copy()
    num_adj_param = 5
    a_param = np.linspace(la, ua, num_adj_param) + (initial_params[adj_param1] + initial_params[adj_param2]) / 2
    size_v_param = np.linspace(0.0005, 0.0015, num_adj_param)
    size_h_param = np.linspace(0.0005, 0.0015, num_adj_param)
    astig = np.linspace(0.0005, 0.0015, num_adj_param)
    steps = []
    for j in range(len(a_param)):
        initial_params[adj_param1] = a_param[j]
        initial_params[adj_param2] = a_param[j]
        size_v_param[j], size_h_param[j], initial_params = focus(initial_params)
        steps.append(sep(initial_params))
        astig[j] = initial_params[1]
    return sep_summary(a_param, size_h_param, steps, option, option_eval, verbose, option_AKB=option_AKB)


def sep_summary(a_param, size_h_param, steps, option='none', option_eval=None, verbose=True, option_AKB=True):
    """What auto_focus_sep forms from its five 'sep' results (:13029-13316): the coma / focus-length
    measures, the printed argmins, and for option='matrix' the scikit-learn line fits, returned per
    option_eval (None otherwise). Host numpy, as the reference."""
    num_adj_param = len(steps)
    arrs = {k: np.zeros((num_adj_param, 3)) for k in ("focus_v0", "focus_h0", "focus_v0_l", "focus_h0_l", "focus_v0_u",
                                                      "focus_h0_u", "std_v0", "std_h0")}
    focus_std_obl1 = np.zeros(num_adj_param)
    focus_std_obl2 = np.zeros(num_adj_param)
    for j, r in enumerate(steps):
        for k in arrs:
            arrs[k][j, :] = r[SEP_OUTPUTS.index(k)]
        focus_std_obl1[j], focus_std_obl2[j] = r[10], r[11]
    focus_v0, focus_h0 = arrs["focus_v0"], arrs["focus_h0"]
    std_v0, std_h0 = arrs["std_v0"], arrs["std_h0"]
    coma_v0 = arrs["focus_v0_l"] - arrs["focus_v0_u"]
    coma_h0 = arrs["focus_h0_l"] - arrs["focus_h0_u"]
    coma_v0_edge = (coma_v0[:, 0] - np.mean(coma_v0, axis=1) + coma_v0[:, 2] - np.mean(coma_v0, axis=1)) / 2.
    coma_h0_edge = (coma_h0[:, 0] - np.mean(coma_h0, axis=1) + coma_h0[:, 2] - np.mean(coma_h0, axis=1)) / 2.
    if verbose:
        print('minimize coma r', a_param[np.argmin(abs(coma_v0[:, 0]))])
        print('minimize coma y', a_param[np.argmin(abs(coma_v0[:, 1]))])
        print('minimize coma g', a_param[np.argmin(abs(coma_v0[:, 2]))])
        print('axial focus distance @V aperture 0', a_param[np.argmin(abs(focus_v0[:, 0] - focus_v0[:, 2]))])
        print('axial focus distance @H aperture 0', a_param[np.argmin(abs(focus_h0[:, 0] - focus_h0[:, 2]))])
        print('focus size std @V aperture 0', a_param[np.argmin(abs(std_v0[:, 0] - std_v0[:, 2]))])
        print('focus size std @H aperture 0', a_param[np.argmin(abs(std_h0[:, 0] - std_h0[:, 2]))])
    focus_len_v0 = focus_v0[:, 0] - np.mean(focus_v0, axis=1) - (focus_v0[:, 2] - np.mean(focus_v0, axis=1))
    coma_h_v0 = ((coma_v0[:, 1]) + (coma_v0[:, 0] + coma_v0[:, 2]) / 2) / 2
    oblique_ast = focus_std_obl1 - focus_std_obl2
    focus_len_h0 = focus_h0[:, 0] - np.mean(focus_h0, axis=1) - (focus_h0[:, 2] - np.mean(focus_h0, axis=1))
    coma_v_h0 = ((coma_h0[:, 1]) + (coma_h0[:, 0] + coma_h0[:, 2]) / 2) / 2
    coma_valance_v0 = coma_v0[:, 0] - np.mean(coma_v0, axis=1) - (coma_v0[:, 2] - np.mean(coma_v0, axis=1))
    coma_valance_h0 = coma_h0[:, 0] - np.mean(coma_h0, axis=1) - (coma_h0[:, 2] - np.mean(coma_h0, axis=1))
    coma_valance_cnt_edg_v0 = coma_v0[:, 1] - np.mean(coma_v0, axis=1) - coma_v0_edge
    coma_valance_cnt_edg_h0 = coma_h0[:, 1] - np.mean(coma_h0, axis=1) - coma_h0_edge
    if option != 'matrix':
        return None
    a = a_param.reshape(-1, 1)
    fits = [_linearfit(a, y, verbose) for y in (oblique_ast, coma_v_h0, coma_h_v0, focus_len_h0, focus_len_v0,
                                                 coma_valance_cnt_edg_h0, coma_valance_cnt_edg_v0, coma_valance_h0,
                                                 coma_valance_v0)]
    (m0, i0, _), (m1, i1, _), (m2, i2, _), (m3, i3, _), (m4, i4, _), (m6, _, _), (m7, _, _), (m8, _, _), (m9, _, _) = fits
    if option_eval == '7':
        return np.array([m0, m3, m4, m6, m7, m8, m9])
    if option_eval == '9':
        return np.array([m0, m1, m2, m3, m4, m6, m7, m8, m9])
    if option_eval == '5':
        return np.array([m0, m3, m4, m8, m9])
    if option_eval == '2':
        return np.array([[m1, m2], [i1, i2]])
    if option_eval == '3':
        return np.array([[m0, m3, m4], [i0, i3, i4]])
    if option_eval == 'KB':
        return np.array([m0, m2, m4])
    if option_eval == '3_intercept':
        return np.array([[m0, m2, m4], [i0, i2, i4]])
    if option_eval == '5coma':
        return np.array([m0, m1, m2, m3, m4])
    if option_eval == '7coma':
        return np.array([m0, m1, m2, m3, m4, m8, m9])
    if option_eval == 'MinimizeH':
        return a_param[np.argmin(size_h_param)]
    if not option_AKB:
        return np.array([m0, m2, m4])
    return np.array([m0, m1, m2, m3, m4, m6, m7, m8, m9])

