"""The on-disk hand-off between the ray tracer and the wave calculation.

saveWaveData (AKB_raytrace_20250312.py:13475-13764) writes, per traced system, a folder holding
  points_source.npy                  the source point (3,)
  points_M1.npy .. points_M4.npy     mirror hit points + area elements (4, N): x, y, z, dS,
                                     dS from calc_dS (:13418-13473) on the (V, H) ray grid
  points_gridImage.npy               an image-plane grid (3, H_f * V_f) around the focus
  points_gridDefocus.npy             the same at the defocused plane (when defocusForWave != 0)
  calculation_conditions.txt         params and grid sizes, "key: value" lines
and the Wavecalc_raytrace_fromData scripts read it back (CPU0402.py:195-380), propagate source ->
M1 -> M2 (-> M3 -> M4) -> image grids with the Huygens sum and save complex_data_<name>.npz
(key 'data'). Here calc_dS runs on the device, the writers reproduce the file set and the
conditions text, read_conditions parses it as the Wavecalc driver does, and run_wave_chain is
that driver's propagation chain on the device (wavecalc.WaveField3D).
"""
import os

import numpy as np
import torch

from . import _lib
from . import device as D


def calc_dS(points, ray_num_V, ray_num_H):
    """Drop-in for calc_dS: area elements (V, H) of a (3, V*H) grid of points, on the device."""
    L = _lib.lib()
    as_torch = isinstance(points, torch.Tensor)
    p = points.to(device=D.device(), dtype=D.F64).contiguous() if as_torch else D.to_dev(points)
    V, H = int(ray_num_V), int(ray_num_H)
    out = torch.empty((V, H), dtype=D.F64, device=p.device)
    _lib.check(L.akb_calc_ds_f64(D.ptr(p), int(p.shape[1]), V, H, D.ptr(out), D.stream_handle()))
    return out if as_torch else out.cpu().numpy()


def downsample_array_3_n(array_3_n, ray_num_V, ray_num_H, downsample_h, downsample_v):
    """downsample_array_3_n (:13336-13356): keep every 2nd column downsample_h // 2 times and
    every 2nd row downsample_v // 2 times. Returns (array, size_v, size_h)."""
    a = np.asarray(array_3_n)
    x = a.reshape(3, ray_num_V, ray_num_H)
    for _ in range(downsample_h // 2):
        x = x[:, :, ::2]
    for _ in range(downsample_v // 2):
        x = x[:, ::2, :]
    return np.ascontiguousarray(x.reshape(3, -1)), x.shape[1], x.shape[2]


def _host(a):
    return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)


def image_grid(detcenter, size_h, size_v, ysize, zsize):
    """The points_gridImage grid of :13644-13662: size_h x size_v points spanning +-ysize, +-zsize
    around the centre of the hits' y / z extent, at x = mean(hits x)."""
    d = _host(detcenter)
    y, z = d[1, :], d[2, :]
    y_grid = np.linspace((np.min(y) + np.max(y)) / 2 - ysize, (np.min(y) + np.max(y)) / 2 + ysize, size_h)
    z_grid = np.linspace((np.min(z) + np.max(z)) / 2 - zsize, (np.min(z) + np.max(z)) / 2 + zsize, size_v)
    yy, zz = np.meshgrid(y_grid, z_grid)
    yf, zf = yy.flatten(), zz.flatten()
    xf = np.full_like(yf, fill_value=np.mean(d[0, :]))
    return np.vstack([xf, yf, zf]), y_grid, z_grid


def save_wave_data(directory, source, mirrors, ray_num_V, ray_num_H, detcenter, detcenter2=None, params=None,
                   ysize=1e-6, zsize=1e-6, defocus_for_wave=0.0, option_AKB=True, option_HighNA=True,
                   option_2mirror=False, option_avrgsplt=False, timestamp="", sizes=None):
    """The file set of saveWaveData (:13506-13654). mirrors: [M1, M2(, M3, M4)] hit points
    (3, V*H) in the reference's naming (M1 = first vertical hyperbola, M2 = horizontal hyperbola,
    M3 / M4 the ellipses). sizes: ((v1, h1), (v2, h2), (vf, hf)) grid shapes of M1 / M3, M2 / M4
    and the detector rows after downsample_array_3_n (default: all ray_num_V x ray_num_H).
    Returns the paths written."""
    os.makedirs(directory, exist_ok=True)
    written = []

    def save(name, arr):
        path = os.path.join(directory, name)
        np.save(path, arr)
        written.append(path)

    (v1, h1), (v2, h2), (vf, hf) = sizes or ((ray_num_V, ray_num_H),) * 3
    src = _host(source)
    save("points_source.npy", src[:, 0] if src.ndim == 2 else src)
    for k, m in enumerate(mirrors):
        pts = _host(m)
        v, h = (v1, h1) if k % 2 == 0 else (v2, h2)
        ds = _host(calc_dS(torch.as_tensor(pts), v, h))
        save(f"points_M{k + 1}.npy", np.vstack((pts, ds.flatten())))
    grid, y_grid, z_grid = image_grid(detcenter, hf, vf, ysize, zsize)
    save("points_gridImage.npy", grid)
    if detcenter2 is not None and np.abs(defocus_for_wave) > 1e-9:
        if option_HighNA:
            span = 2e-7 + defocus_for_wave * 0.082 * 2
        else:
            span = 2e-7 + defocus_for_wave * 0.01 * 2
        grid2, _, _ = image_grid(detcenter2, hf, vf, span, span)
        save("points_gridDefocus.npy", grid2)
    p = np.zeros(26) if params is None else np.asarray(params)
    path = os.path.join(directory, "calculation_conditions.txt")
    with open(path, "w") as f:
        f.write("Conditions\n")
        f.write("====================\n")
        f.write(f"time: {timestamp}\n")
        f.write(f"params 0-1: {p[0:2]}\n")
        f.write(f"params 2-7: {p[2:8]}\n")
        f.write(f"params 8-13: {p[8:14]}\n")
        f.write(f"params 14-19: {p[14:20]}\n")
        f.write(f"params 20-26: {p[20:26]}\n")
        f.write(f"grid pitch_y: {y_grid[1] - y_grid[0]}\n")
        f.write(f"grid pitch_z: {z_grid[1] - z_grid[0]}\n")
        f.write(f"grid size_y: {np.max(y_grid) - np.min(y_grid)}\n")
        f.write(f"grid size_z: {np.max(z_grid) - np.min(z_grid)}\n")
        f.write(f"grid pix_y: {hf}\n")
        f.write(f"grid pix_z: {vf}\n")
        f.write(f"grid pix_H1: {h1}\n")
        f.write(f"grid pix_V1: {v1}\n")
        f.write(f"grid pix_H2: {h2}\n")
        f.write(f"grid pix_V2: {v2}\n")
        f.write(f"option_AKB: {option_AKB}\n")
        f.write(f"option_HighNA: {option_HighNA}\n")
        f.write(f"defocusForWave: {defocus_for_wave}\n")
        f.write(f"calc both mirrors?: {option_2mirror}\n")
        f.write(f"option_avrgsplt: {option_avrgsplt}\n")
        f.write("====================\n")
    written.append(path)
    return written


def read_conditions(folder):
    """calculation_conditions.txt read as the Wavecalc driver reads it (CPU0402.py:208-236)."""
    c = {}
    with open(os.path.join(folder, "calculation_conditions.txt")) as f:
        for line in f:
            v = line.split(":")[1].strip() if ":" in line else ""
            if "grid pix_y:" in line:
                c["pix_y"] = c["ray_num_H1"] = c["ray_num_H2"] = int(v)
            elif "grid pix_z:" in line:
                c["pix_z"] = c["ray_num_V1"] = c["ray_num_V2"] = int(v)
            elif "grid pix_H:" in line:
                c["ray_num_H1"] = c["ray_num_V2"] = int(v)
            elif "grid pix_V:" in line:
                c["ray_num_V1"] = c["ray_num_H2"] = int(v)
            elif "grid pix_H1:" in line:
                c["ray_num_H1"] = int(v)
            elif "grid pix_V1:" in line:
                c["ray_num_V1"] = int(v)
            elif "grid pix_H2:" in line:
                c["ray_num_H2"] = int(v)
            elif "grid pix_V2:" in line:
                c["ray_num_V2"] = int(v)
            elif "option_AKB:" in line:
                c["option_AKB"] = v.lower() == "true"
            elif "option_HighNA:" in line:
                c["option_HighNA"] = v.lower() == "true"
    return c


def load_npz_data(filename):
    """load_npz_data (CPU0402.py:173-187): the 'data' array of an .npz, or None when the file does not
    exist. Loaded without pickle (numpy's default)."""
    if os.path.exists(filename):
        with np.load(filename) as data:
            return data["data"]
    return None


def run_wave_chain(folder, out_dir=None, files=("points_source.npy", "points_M1.npy", "points_M2.npy",
                                                "points_gridImage.npy", "points_gridDefocus.npy"), resume_dir=".",
                   resumed=None):
    """The Wavecalc_raytrace_fromData driver (CPU0402.py:186-380) on the device: source -> M1 ->
    M2 (-> M3 -> M4) -> image grid (scaled x2 about its mean) and the second image grid, saving
    complex_data_<name>.npz (key 'data') into out_dir. Returns {name: field (numpy complex128)}.

    Stage resume, as the driver does (:261-269, :281-290, and M3 / M4): a mirror stage whose
    complex_data_M<k>.npz is found in resume_dir (the driver looks in the working directory, the
    default here) takes that field instead of propagating, and it is not written again; None
    switches resuming off (resumed, a list, receives the names of the stages taken from files). The
    image stages are always computed."""
    from .wavecalc import WaveField3D
    cond = read_conditions(folder)
    akb = cond.get("option_AKB", True)
    wl = 13.5e-9 if cond.get("option_HighNA", True) else 13.5e-9 * 1e-1
    load = lambda name: np.load(os.path.join(folder, name))  # noqa: E731
    source = load(files[0])
    fields = {}

    def store(name, u):
        fields[name] = np.asarray(u)
        if out_dir is not None:
            os.makedirs(out_dir, exist_ok=True)
            np.savez_compressed(os.path.join(out_dir, f"complex_data_{name}.npz"), data=fields[name])

    src = WaveField3D(1, wl, 1, 1)
    src.u[0] = 1.0
    src.setdata(source.reshape(3, 1))
    src.set_ds(np.ones(1))
    chain = ["points_M1.npy", "points_M2.npy"] + (["points_M3.npy", "points_M4.npy"] if akb else [])
    dims = [(cond["ray_num_H1"], cond["ray_num_V1"]), (cond["ray_num_H2"], cond["ray_num_V2"])] * 2
    prev = src
    resumed = [] if resumed is None else resumed
    for k, fname in enumerate(chain):
        pts = load(fname)
        f = WaveField3D(pts.shape[1], wl, *dims[k])
        f.setdata(pts)
        data = load_npz_data(os.path.join(resume_dir, f"complex_data_M{k + 1}.npz")) if resume_dir is not None else None
        if data is not None:
            if data.shape != (pts.shape[1],):
                raise ValueError(f"complex_data_M{k + 1}.npz holds {data.shape} values for {pts.shape[1]} points")
            f.u = np.asarray(data, dtype=np.complex128)
            fields[f"M{k + 1}"] = f.u
            resumed.append(f"M{k + 1}")
        else:
            f.forward_propagation(prev)
            store(f"M{k + 1}", f.u)
        f.set_ds(pts[3, :])
        prev = f
    img = load(files[3]).copy()
    mean = [np.mean(img[0, :]), np.mean(img[1, :]), np.mean(img[2, :])]
    for r in range(3):
        img[r, :] = (img[r, :] - mean[r]) * 2. + mean[r]
    g = WaveField3D(img.shape[1], wl, cond["pix_y"], cond["pix_z"])
    g.setdata(img)
    g.forward_propagation(prev)
    store("Image", g.u)
    if os.path.exists(os.path.join(folder, files[4])):
        img2 = load(files[4]).copy()
        mean2 = [np.mean(img2[0, :]), np.mean(img2[1, :]), np.mean(img2[2, :])]
        for r in range(3):
            img2[r, :] = (img2[r, :] - mean2[r]) + mean2[r]
        g2 = WaveField3D(img2.shape[1], wl, cond["pix_y"], cond["pix_z"])
        g2.setdata(img2)
        g2.forward_propagation(prev)
        store("Image2", g2.u)
    return fields


def two_pass_trace(b, n, mode="wave"):
    """The two-pass trace every resampled mode of plot_result_debug shares ('sep', 'wave', 'ray',
    'ray_wave': :2694-2845 pass 1, :2849-2879 the equal-angle resample, :2881-2905 pass 2) for the
    built system b on an n x n grid: pass 1 traces only the resample's picks' exit slopes (the
    full pass 1 is still traced for its flags), the host resamples with numpy's arctan / tan and
    the C interp1d, pass 2 keeps every mirror's hits, the exit directions and the detector hits on
    coeffs_det = (g = 1, j = -(s2f_middle + defocus)). Returns device tensors (hits (4, 3, n^2),
    exit directions, detcenter). A flagged pass 2 takes the drop-in primitives stage by stage,
    which apply the reference's all-NaN / passthrough rules."""
    from . import geometry as G
    from . import primitives as P
    from .trace import grid_dirs, staged_chain, trace_chain
    from .wavefront import AngleRange, resample, sample_plan
    dev = D.device()
    mir = G.mirrors_of(b)
    rand_h = AngleRange(**b["angle_h"]).table(n)
    rand_v = AngleRange(**b["angle_v"]).table(n)
    th = torch.from_numpy(np.tan(rand_h)).to(dev)
    tv = torch.from_numpy(np.tan(rand_v)).to(dev)
    hb, he, col = sample_plan(n)
    r1 = trace_chain(mir, tan_h=th, tan_v=tv, src=b["source"], want=(), samples=(hb, he, col))
    f1 = int(r1.flags.item())
    if f1:
        raise _lib.AKBError(f"pass 1 of the '{mode}' trace flagged 0x{f1:x} (a miss or zero norm: the reference's "
                            "all-NaN rays cannot be resampled)")
    s = r1.extra["samples"].cpu().numpy()
    rand_h2, rand_v2 = resample(np.arctan(s[:he - hb]), np.arctan(s[he - hb:]), rand_h, rand_v)
    th2 = torch.from_numpy(np.tan(rand_h2)).to(dev)
    tv2 = torch.from_numpy(np.tan(rand_v2)).to(dev)
    det1 = b["det1"][6:10]
    r2 = trace_chain(mir, tan_h=th2, tan_v=tv2, src=b["source"], want=("hits", "dir_out", "det"), det_ghij=det1)
    N = n * n
    if int(r2.flags.item()):
        src = torch.tensor(b["source"], dtype=D.F64, device=dev).reshape(3, 1).expand(3, N).contiguous()
        hits, refl, _ = staged_chain(mir, grid_dirs(th2, tv2), src)
        hits = torch.stack(hits)
        det = P.plane_ray_intersection(b["det1"], refl, hits[-1])
        return hits, refl, det
    return r2.hits, r2.dir_out, r2.det


def plot_result_wave(params, ray_num, *, defocus_for_wave=1e-3, option_set=True, source_shift=(0.0, 0.0, 0.0),
                     as_torch=False):
    """plot_result_debug(params, 'wave') (AKB_raytrace_20250312.py:2675-2905, :3510-3561) on the
    device for the AKB system built from params (geometry.build_akb), on a ray_num x ray_num grid:
    pass 1, the equal-angle resample (host numpy arctan / tan and the C interp1d, as RayWave), pass
    2 with every mirror's hits, then the 'wave' tilt - theta from np.mean (not nanmean) of the exit
    slopes' arctan, every mirror grid and the source rotated about np.mean(detcenter, axis=1) -
    the re-intersected detector and, when |defocus_for_wave| > 1e-9, the defocused one. Returns the
    reference's tuple: (source, vmirr_hyp, hmirr_hyp, vmirr_ell, hmirr_ell, detcenter[, detcenter2],
    ray_num_H, ray_num_V, vmirr_norm, hmirr_norm, vmirr2_norm, hmirr2_norm, vec0to1, vec1to2,
    vec2to3, vec3to4), or np.inf where the reference returns np.inf."""
    from . import geometry as G
    from . import primitives as P
    from .reduce import means_to_host, np_sum
    b = G.build_akb(params, source_shift=source_shift, option_set=option_set)
    if not isinstance(b, dict):
        return b
    n = int(ray_num)
    dev = D.device()
    hits, refl, det = two_pass_trace(b, n, "wave")
    # theta from the exit slopes (:3516-3517), numpy on the host as the reference
    ang = refl.cpu().numpy()
    theta_y = -np.mean(np.arctan(ang[2, :] / ang[0, :]))
    theta_z = np.mean(np.arctan(ang[1, :] / ang[0, :]))
    (focus,) = means_to_host([np_sum(det)])  # np.mean(detcenter, axis=1), numpy's order on the device
    source0 = torch.zeros((3, 1), dtype=D.F64, device=dev)
    refl_rot = P.rotate_vectors(refl, -theta_y, -theta_z)
    rot = [P.rotate_points(hits[k], focus, -theta_y, -theta_z) for k in range(4)]
    src_rot = P.rotate_points(source0, focus, -theta_y, -theta_z)
    vmirr_hyp, vmirr_ell, hmirr_ell, hmirr_hyp = rot
    detcenter = P.plane_ray_intersection(b["det1"], refl_rot, hmirr_hyp)
    vec0to1 = P.normalize_vector(vmirr_hyp - src_rot)
    vec1to2 = P.normalize_vector(vmirr_ell - vmirr_hyp)
    vec2to3 = P.normalize_vector(hmirr_ell - vmirr_ell)
    vec3to4 = P.normalize_vector(hmirr_hyp - hmirr_ell)
    vec4to5 = P.normalize_vector(detcenter - hmirr_hyp)
    norms = [P.normalize_vector((-b_ + a_) / 2) for a_, b_ in
             ((vec0to1, vec1to2), (vec1to2, vec2to3), (vec2to3, vec3to4), (vec3to4, vec4to5))]
    out = [src_rot, vmirr_hyp, hmirr_hyp, vmirr_ell, hmirr_ell, detcenter]
    if np.abs(defocus_for_wave) > 1e-9:
        c2 = np.zeros(10)
        c2[6] = 1
        c2[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]) + defocus_for_wave)
        out.append(P.plane_ray_intersection(c2, refl_rot, hmirr_hyp))
    out += [n, n] + norms + [vec0to1, vec1to2, vec2to3, vec3to4]
    if as_torch:
        return tuple(out)
    return tuple(x.cpu().numpy() if isinstance(x, torch.Tensor) else x for x in out)


def kb_wave(params, ray_num, *, defocus_for_wave=1e-3, source_shift=(0.0, 0.0, 0.0), designparams=None,
            as_torch=False):
    """KB_debug(params, na_ratio_h, na_ratio_v, 'wave') (AKB_raytrace_20250312.py:10948-11054,
    :11629-11701; option_rotate True, option_avrgsplt False) on the device for the KB pair of
    geometry.build_kb on a ray_num x ray_num grid: pass 1, reset_p0's equal-angle resample, pass 2,
    the np.mean tilt, both mirror grids and the (unshifted) source rotated about
    np.mean(detcenter, axis=1), the re-intersected detector and, when |defocus_for_wave| > 1e-9, the
    defocused one. Returns the reference's tuple: (source, vmirr_hyp, hmirr_hyp, detcenter[,
    detcenter2], ray_num_H, ray_num_V, vmirr_norm, hmirr_norm, vec0to1, vec1to2), or np.inf where
    the reference returns np.inf."""
    from . import geometry as G
    from . import primitives as P
    from .reduce import means_to_host, np_sum
    b = G.build_kb(params, source_shift=source_shift, designparams=designparams)
    if not isinstance(b, dict):
        return b
    n = int(ray_num)
    dev = D.device()
    hits, refl, det = two_pass_trace(b, n, "wave")
    ang = refl.cpu().numpy()
    theta_y = -np.mean(np.arctan(ang[2, :] / ang[0, :]))  # :11634-11635
    theta_z = np.mean(np.arctan(ang[1, :] / ang[0, :]))
    (focus,) = means_to_host([np_sum(det)])  # np.mean(detcenter, axis=1) of pass 2's hits (:11639)
    source0 = torch.zeros((3, 1), dtype=D.F64, device=dev)
    refl_rot = P.rotate_vectors(refl, -theta_y, -theta_z)
    hmirr = P.rotate_points(hits[1], focus, -theta_y, -theta_z)
    src_rot = P.rotate_points(source0, focus, -theta_y, -theta_z)
    vmirr = P.rotate_points(hits[0], focus, -theta_y, -theta_z)
    detcenter = P.plane_ray_intersection(b["det1"], refl_rot, hmirr)  # :11683-11686
    vec0to1 = P.normalize_vector(vmirr - src_rot)
    vec1to2 = P.normalize_vector(hmirr - vmirr)
    vec2to3 = P.normalize_vector(detcenter - hmirr)
    vmirr_norm = P.normalize_vector((-vec1to2 + vec0to1) / 2)
    hmirr_norm = P.normalize_vector((-vec2to3 + vec1to2) / 2)
    out = [src_rot, vmirr, hmirr, detcenter]
    if np.abs(defocus_for_wave) > 1e-9:
        c2 = np.zeros(10)
        c2[6] = 1
        c2[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]) + defocus_for_wave)
        out.append(P.plane_ray_intersection(c2, refl_rot, hmirr))
    out += [n, n, vmirr_norm, hmirr_norm, vec0to1, vec1to2]
    if as_torch:
        return tuple(out)
    return tuple(x.cpu().numpy() if isinstance(x, torch.Tensor) else x for x in out)


def saveWaveData(initial_params, ysize=1e-6, zsize=1e-6, *, ray_num_H=65, ray_num_V=None, directory=None,
                 defocus_for_wave=1e-3, downsample=(0, 0, 0, 0, 0, 0), option_set=True, option_HighNA=True,
                 option_2mirror=True, option_avrgsplt=False, timestamp=None, option_AKB=True, kb_design=None):
    """saveWaveData (AKB_raytrace_20250312.py:13475-13764) for the AKB system, without its final
    sys.exit(): the 'wave' run (plot_result_wave), downsample_array_3_n of every grid when the grid
    is odd (:13489-13497, factors (h1, v1, h2, v2, h_f, v_f) = the module's downsample_* flags), the
    area elements on the device, and the file set into `directory` (default output_<timestamp>,
    as the reference). Returns the directory. The module flags the reference reads (wave_num_H /
    wave_num_V, defocusForWave, option_HighNA, option_2mirror, option_avrgsplt, option_set) are
    keyword arguments here; install() passes the module's live values. option_AKB False: KB_debug's
    pair (kb_wave; kb_design = the module's KBdesign_7params) and its two-mirror file set."""
    from datetime import datetime
    ray_num_V = ray_num_H if ray_num_V is None else ray_num_V
    if ray_num_V != ray_num_H:
        raise ValueError("the 'wave' grid is square (ray_num = wave_num_H, :1890-1893, :10412-10415)")
    two = np.abs(defocus_for_wave) > 1e-9
    if option_AKB:
        r = plot_result_wave(initial_params, ray_num_H, defocus_for_wave=defocus_for_wave, option_set=option_set)
    else:
        r = kb_wave(initial_params, ray_num_H, defocus_for_wave=defocus_for_wave, designparams=kb_design)
    if not isinstance(r, tuple):
        raise TypeError("cannot unpack non-iterable float object")  # the reference unpacks np.inf
    if option_AKB:
        source, vmirr_hyp, hmirr_hyp, vmirr_ell, hmirr_ell, detcenter = r[:6]
        detcenter2 = r[6] if two else None
    else:
        source, vmirr_hyp, hmirr_hyp, detcenter = r[:4]
        vmirr_ell = hmirr_ell = None
        detcenter2 = r[4] if two else None
    if ray_num_H % 2 != 1:
        # the reference only sets the grid sizes inside its odd-grid branch
        raise NameError("name 'size_v1' is not defined")
    h1, v1, h2, v2, hf, vf = downsample
    vmirr_hyp, size_v1, size_h1 = downsample_array_3_n(vmirr_hyp, ray_num_V, ray_num_H, h1, v1)
    hmirr_hyp, size_v2, size_h2 = downsample_array_3_n(hmirr_hyp, ray_num_V, ray_num_H, h2, v2)
    detcenter, size_v_f, size_h_f = downsample_array_3_n(detcenter, ray_num_V, ray_num_H, hf, vf)
    if option_AKB:
        vmirr_ell, _, _ = downsample_array_3_n(vmirr_ell, ray_num_V, ray_num_H, h1, v1)
        hmirr_ell, _, _ = downsample_array_3_n(hmirr_ell, ray_num_V, ray_num_H, h2, v2)
    if two:
        detcenter2, _, _ = downsample_array_3_n(detcenter2, ray_num_V, ray_num_H, hf, vf)
    timestamp = timestamp or datetime.now().strftime('%Y%m%d_%H%M%S')
    directory = directory or f"output_{timestamp}"
    mirrors = [vmirr_hyp, hmirr_hyp] + ([vmirr_ell, hmirr_ell] if option_AKB else [])
    save_wave_data(directory, source, mirrors, ray_num_V, ray_num_H,
                   detcenter, detcenter2, params=initial_params, ysize=ysize, zsize=zsize,
                   defocus_for_wave=defocus_for_wave, option_AKB=bool(option_AKB), option_HighNA=option_HighNA,
                   option_2mirror=option_2mirror, option_avrgsplt=option_avrgsplt, timestamp=timestamp,
                   sizes=((size_v1, size_h1), (size_v2, size_h2), (size_v_f, size_h_f)))
    return directory
