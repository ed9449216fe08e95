"""Hot-path slice of the reference's trace drivers, restated over the oracle primitives.
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

What plot_result_debug (AKB_raytrace_20250312.py:1326, Wolter 3-1) and KB_debug (:9742) do with
a ray grid once their mirror coefficients are set up:

  grid      rand_p0h/rand_p0v = linspace(endpoints) - offset; phai0[:, iv*n + ih] =
            normalize(1, tan(rand_p0h[ih]), tan(rand_p0v[iv]))               :2694-2717
  pass 1    mirror chain (intersect -> normal -> reflect), detector plane     :2770-2845
  resample  equal exit-angle grid from interp1d on the middle row / column    :2849-2879
  pass 2    mirror chain again + segment lengths dist0to1 ...                  :2881-2905
  tilt      theta from nanmean(arctan), rotate direction and last hit about
            mean(detcenter), detector re-intersected                          :3583-3601
  ray_wave  detcenter2 at +defocusWave, totalDist, DistError, Sph, Wave2       :3611-3677

Geometry comes from tests/golden/akb_geometry.json / kb_geometry.json (recorded from the
reference). Means use numpy itself (the reference's own arithmetic).
"""
import numpy as np
from scipy.interpolate import interp1d

import oracle as O


def angle_tables(geom, n):
    """rand_p0h, rand_p0v and their tangents exactly as the driver forms them (:2695-2717):
    np.tan on the H array once, np.tan on each V angle as a scalar per row."""
    h, v = geom["angle_h"], geom["angle_v"]
    rand_h = np.linspace(h["start"], h["stop"], n) - np.float64(h["offset"])
    rand_v = np.linspace(v["start"], v["stop"], n) - np.float64(v["offset"])
    tan_h = np.tan(rand_h)
    tan_v = np.array([np.tan(x) for x in rand_v], dtype=np.float64)
    return rand_h, rand_v, tan_h, tan_v


def grid_dirs(tan_h, tan_v):
    nh, nv = tan_h.shape[0], tan_v.shape[0]
    phai0 = np.zeros((3, nh * nv))
    phai0[0] = 1.0
    phai0[1] = np.tile(tan_h, nv)
    phai0[2] = np.repeat(tan_v, nh)
    return O.normalize_vector(phai0)


def chain(mirrors, dirs, src, with_segments=False):
    """Sequential mirror chain with the reference's stage semantics. Returns (hits, dirs_after,
    segments) where hits[k] is the hit on mirror k."""
    hits, segs = [], []
    ray, org = dirs, src
    for m in mirrors:
        p = O.mirr_ray_intersection(m["coeffs"], ray, org, negative=m["negative"])
        if with_segments:
            segs.append(O.seglen(org, p))
        ray = O.reflect_ray(ray, O.norm_vector(m["coeffs"], p))
        org = p
        hits.append(p)
    return hits, ray, segs


def sample_indices(n_h, n_v):
    """The middle column / middle row picks of the equal-angle resample (:2851-2856):
    original_array[round((n-1)/2)::n] and crop(round(n(n-1)/2), round(n(n+1)/2), 1)."""
    col = round((n_h - 1) / 2)
    v_idx = np.arange(col, n_h * n_v, n_h)
    start = round(n_h * (n_v - 1) / 2)
    end = round(n_h * (n_v + 1) / 2)
    h_idx = np.arange(start, end)
    return col, v_idx, start, end, h_idx


def resample_tables(refl, rand_h, rand_v, n_h, n_v):
    """:2857-2870 — new rand_p0v/rand_p0h so the exit angles are equally spaced."""
    _, v_idx, _, _, h_idx = sample_indices(n_h, n_v)
    angle_h = np.arctan(refl[1, h_idx] / refl[0, h_idx])
    angle_v = np.arctan(refl[2, v_idx] / refl[0, v_idx])
    return resample_from_angles(angle_h, angle_v, rand_h, rand_v)


def resample_from_angles(angle_h_sep, angle_v_sep, rand_h, rand_v):
    out_v = np.linspace(angle_v_sep[0], angle_v_sep[-1], len(angle_v_sep))
    out_h = np.linspace(angle_h_sep[0], angle_h_sep[-1], len(angle_h_sep))
    new_v = interp1d(angle_v_sep, rand_v, kind="linear")(out_v)
    new_h = interp1d(angle_h_sep, rand_h, kind="linear")(out_h)
    return new_h, new_v


def tilt(refl, last_hit, det_pre, det_ghij):
    """:3583-3601 (option_tilt, non-'ray' branch)."""
    theta_y = -np.nanmean(np.arctan(refl[2, :] / refl[0, :]))
    theta_z = np.nanmean(np.arctan(refl[1, :] / refl[0, :]))
    refl_rot = O.rotate_vectors(refl, -theta_y, -theta_z)
    focus_apprx = np.mean(det_pre, axis=1)
    pt_rot = O.rotate_points(last_hit, focus_apprx, -theta_y, -theta_z)
    coeffs = np.zeros(10)
    coeffs[6:10] = det_ghij
    det = O.plane_ray_intersection(coeffs, refl_rot, pt_rot)
    return refl_rot, pt_rot, det, (theta_y, theta_z, focus_apprx)


def akb_ray_wave(geom, n, source=None):
    """The 'ray_wave' hot path of the Wolter 3-1 plot_result_debug on an n x n grid, up to the
    griddata inputs (:3689); with a 2-mirror geometry KB_debug's 'wave' trace and OPD (:11629-11700).
    Returns a dict of the intermediate arrays."""
    src = np.zeros((3, n * n)) if source is None else source
    mirrors = geom["mirrors"]
    det1 = np.zeros(10)
    det1[6:10] = geom["det1"][6:10]
    det2 = np.zeros(10)
    det2[6:10] = geom["det2"][6:10]
    rand_h, rand_v, tan_h, tan_v = angle_tables(geom, n)
    dirs = grid_dirs(tan_h, tan_v)
    _, r4, _ = chain(mirrors, dirs, src)
    new_h, new_v = resample_tables(r4, rand_h, rand_v, n, n)
    tan_h2 = np.tan(new_h)
    tan_v2 = np.array([np.tan(x) for x in new_v], dtype=np.float64)
    dirs2 = grid_dirs(tan_h2, tan_v2)
    hits, r4, segs = chain(mirrors, dirs2, src, with_segments=True)
    det_pre = O.plane_ray_intersection(det1, r4, hits[-1])
    r4r, p4r, det, (ty, tz, fa) = tilt(r4, hits[-1], det_pre, geom["det1"][6:10])
    det_2 = O.plane_ray_intersection(det2, r4r, p4r)
    d4 = O.seglen(p4r, det)
    mirr = segs[0]
    for sg in segs[1:]:  # left to right, as the drivers write dist0to1 + dist1to2 + ... (K = 4 or 2)
        mirr = mirr + sg
    total = mirr + d4
    dist_err = (total - np.nanmean(total)) * 1e9
    d4b = O.seglen(p4r, det_2)
    total2 = mirr + d4b
    dist_err2 = (total2 - np.nanmean(total2)) * 1e9
    mean_focus = np.nanmean(det, axis=1)
    sph = O.seglen(np.broadcast_to(mean_focus[:, None], det_2.shape).copy(), det_2) * 1e9
    wave2 = dist_err2 - sph
    return dict(tan_h=tan_h, tan_v=tan_v, tan_h2=tan_h2, tan_v2=tan_v2, dirs2=dirs2, hits=hits, segs=segs,
                r4=r4, det_pre=det_pre, r4_rot=r4r, p4_rot=p4r, detcenter=det, detcenter2=det_2,
                theta_y=ty, theta_z=tz, focus_apprx=fa, total=total, total2=total2, dist_err=dist_err,
                dist_err2=dist_err2, mean_focus=mean_focus, sph=sph, wave2=wave2)


def kb_wave(geom, n):
    """KB_debug 'wave' trace (:10948-10997 plus the reset_p0 resample :11010-11054): two
    ellipses, pass 1, equal-angle resample, pass 2 to the detector."""
    src = np.zeros((3, n * n))
    h, v = geom["angle_h"], geom["angle_v"]
    rand_h = np.linspace(h["start"], h["stop"], n) - np.float64(h["offset"])
    rand_v = np.linspace(v["start"], v["stop"], n) - np.float64(v["offset"])
    tan_h = np.tan(rand_h)
    tan_v = np.array([np.tan(x) for x in rand_v])
    det = np.zeros(10)
    det[6:10] = geom["det1"][6:10]
    hits1, r2, _ = chain(geom["mirrors"], grid_dirs(tan_h, tan_v), src)
    new_h, new_v = resample_tables(r2, rand_h, rand_v, n, n)
    tan_h2 = np.tan(new_h)
    tan_v2 = np.array([np.tan(x) for x in new_v])
    dirs2 = grid_dirs(tan_h2, tan_v2)
    hits2, r2b, _ = chain(geom["mirrors"], dirs2, src)
    det2 = O.plane_ray_intersection(det, r2b, hits2[-1])
    return dict(hits1=hits1, refl1=r2, dirs2=dirs2, hits2=hits2, refl2=r2b, det=det2)
