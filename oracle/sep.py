"""compare_sep / optimize_min_index restated on the CPU — TEST INFRASTRUCTURE ONLY (see
oracle/__init__.py). Pinned by tests/golden/akb_sep.npz (make_golden_sep.py).

AKB_raytrace_20250312.py:
  optimize_min_index      :9174-9217   100-point np.linspace grid, np.argmin, the range shrunk
                                       by 0.1 about the best point until narrower than 1e-13
  create_func_to_minimize :9219-9239   plane x = -a (coeffs_det[9] = a, written into the caller's
                                       array) intersected with a subset of the rays
  create_evaluation_fn    :9241-9265   sqrt(np.std(z)**2 + np.std(y)**2)
  compare_sep             :9267-9560   twenty such searches over row / column / partial /
                                       diagonal subsets, then the mean hit positions on the
                                       last searched plane
"""
import numpy as np

from . import plane_ray_intersection


def subsets(ray_num, n_rays):
    """The twenty index sets of compare_sep in call order (:9278-9304, :9334-9541)."""
    n = int(ray_num)
    full = list(range(n * n))
    v_r = full[::n]
    v_y = full[round((n - 1) / 2)::n]
    v_g = full[n - 1::n]
    h_r = list(range(n + 1))[0:n:1]
    a, b = round(n * (n - 1) / 2), round(n * (n + 1) / 2)
    h_y = list(range(b + 1))[a:b:1]
    h_g = list(range(n * n + 1))[n * n - n:n * n:1]
    t = {k: len(v) * 2 // 3 for k, v in (("vr", v_r), ("vy", v_y), ("vg", v_g), ("hr", h_r), ("hy", h_y),
                                           ("hg", h_g))}
    obl1 = np.arange(n - 1, n_rays, n - 1)[:-1]
    obl2 = np.arange(0, n_rays, n + 1)
    return [h_r, h_y, h_g, v_r, v_y, v_g,
            h_r[:t["hr"]], h_y[:t["hy"]], h_g[:t["hg"]], v_r[:t["vr"]], v_y[:t["vy"]], v_g[:t["vg"]],
            h_r[:-t["hr"]], h_y[:-t["hy"]], h_g[:-t["hg"]], v_r[:-t["vr"]], v_y[:-t["vy"]], v_g[:-t["vg"]],
            obl1, obl2]


def optimize_min_index(func, x_min, x_max, num_steps=100, shrink_factor=0.1, max_attempts=20, tolerance=1e-13):
    attempt = 0
    best_x = min_y = None
    while attempt < max_attempts:
        x_values = np.linspace(x_min, x_max, num_steps)
        y_values = np.array([func(x) for x in x_values])
        i = np.argmin(y_values)
        best_x, min_y = x_values[i], y_values[i]
        delta_x = (x_max - x_min) * shrink_factor
        x_min = best_x - delta_x / 2
        x_max = best_x + delta_x / 2
        if (x_max - x_min) < tolerance and x_max - x_min > 1e-16:
            break
        attempt += 1
    return best_x, min_y


def compare_sep(rays, points, coeffs_det0, ray_num, region=1e-4, widesearch=False):
    """The reference's twelve outputs; coeffs_det0 is updated in place as the reference does."""
    w = 1e-1 if widesearch else 1e-2
    x_min, x_max = coeffs_det0[9] - w, coeffs_det0[9] + w

    def func(idx):
        sub_r, sub_p = rays[:, idx], points[:, idx]

        def f(a):
            coeffs_det0[6] = 1.
            coeffs_det0[9] = a
            det = plane_ray_intersection(coeffs_det0, sub_r, sub_p)
            sv, sh = np.std(det[2, :]), np.std(det[1, :])
            return np.sqrt(sv**2 + sh**2)
        return f

    res = [optimize_min_index(func(idx), x_min=x_min, x_max=x_max) for idx in subsets(ray_num, rays.shape[1])]
    foc = [r[0] for r in res]
    std = [r[1] for r in res]
    n = int(ray_num)
    det = plane_ray_intersection(coeffs_det0, rays, points)
    d2r, d2y, d2g = det[:, ::n], det[:, round((n - 1) / 2)::n], det[:, n - 1::n]
    d1r = det[:, :n]
    d1y = det[:, round(n * (n - 1) / 2): round(n * (n + 1) / 2)]
    d1g = det[:, -n:]
    pos_v0 = np.array([[np.mean(d1r, axis=1)], [np.mean(d1y, axis=1)], [np.mean(d1g, axis=1)]])
    pos_h0 = np.array([[np.mean(d2r, axis=1)], [np.mean(d2y, axis=1)], [np.mean(d2g, axis=1)]])
    return (np.array(foc[0:3]), np.array(foc[3:6]), pos_v0, pos_h0, np.array(std[0:3]), np.array(std[3:6]),
            np.array(foc[6:9]), np.array(foc[9:12]), np.array(foc[12:15]), np.array(foc[15:18]), foc[18], foc[19])
