"""Batched focus searches on the device: the 'test' trace of
plot_result_debug and the auto_focus_NA / calc_FoC loops that call it hundreds of times.

plot_result_debug(params, 'test') (AKB_raytrace_20250312.py:1326-4496) builds its system from
params (geometry.build_akb), traces a 53 x 53 grid once through the four mirrors (:2770-2821),
intersects a detector plane x = s2f_middle + params[0] (:2842-2845), tilts the rays by the mean
exit angles and re-intersects (:3565-3601), and returns the hits. auto_focus_NA (:12746-12895)
sweeps params[0] over 100 values per attempt, taking np.std of the detector hits each time;
params[0] only moves the detector plane, so every sweep is one system against 100 planes.

Here a sweep is:
  TestTrace        the system built once per distinct params[1:] (the mirrors do not depend on
                   params[0]) and traced once - akb_trace_chain_batch_f64, any number of systems
                   in one launch; the tilt angles np.nanmean(np.arctan(...)) and the rotation
                   matrices are formed by numpy on the host from the traced exit directions,
                   exactly as the reference forms them (numpy's SIMD arctan has no bitwise device
                   equivalent, and it is one 53 x 53 array per system)
  focus_eval       akb_focus_eval_f64: every (system, plane) pair in one launch - detector hits,
                   np.mean focus, rotation in dgemm order, re-intersection, np.std of y and z in
                   numpy's summation order
so the spot sizes, the argmins auto_focus_NA takes over them and its answer are the reference's
bit for bit (tests/golden/akb_autofocus.npz). A flagged trace (a miss or zero norm) takes the
drop-in primitives stage by stage, which apply the reference's all-NaN / passthrough rules.

KB_debug(params, na_ratio_h, na_ratio_v, 'test') (:9742-12726) - the KB pair auto_focus_NA sweeps
when option_AKB is False - is kb_test: geometry.build_kb's two ellipses through the same batched
trace and evaluation, tilted always and by np.mean (not nanmean) of the exit angles
(tests/golden/kb_build.npz).
"""
import numpy as np
import torch

from . import _lib
from . import device as D
from . import geometry as G
from . import primitives as P
from .trace import staged_chain
from .wavefront import AngleRange


def _tables(built, n):
    """tan(rand_p0h), tan(rand_p0v) of :2695-2715 (host numpy, as the reference)."""
    th = np.tan(AngleRange(**built["angle_h"]).table(n))
    tv = np.tan(AngleRange(**built["angle_v"]).table(n))
    return th, tv


class TracedSystems:
    """S systems traced on an n x n grid: exit directions and last hits (S, 3, n^2) on the device,
    their tilt rotations (S, 18) and detector-plane offsets s2f_middle."""

    def __init__(self, builts, ray_num=53, want_hits=False, tilt=True, theta_mean="nanmean"):
        L = _lib.lib()
        if theta_mean not in ("nanmean", "mean"):
            raise ValueError("theta_mean is 'nanmean' (plot_result_debug) or 'mean' (KB_debug)")
        self.theta_mean = theta_mean
        self.dev = D.device()
        self.builts = list(builts)
        S = len(self.builts)
        n = int(ray_num)
        N = n * n
        self.S, self.n, self.N = S, n, N
        self.dir = torch.empty((S, 3, N), dtype=D.F64, device=self.dev)
        self.pt = torch.empty((S, 3, N), dtype=D.F64, device=self.dev)
        K = len(self.builts[0]["mirrors"])
        if any(len(b["mirrors"]) != K for b in self.builts):
            raise ValueError("every system of a batch has the same number of mirrors")
        self.hits = torch.empty((S, K, 3, N), dtype=D.F64, device=self.dev) if want_hits else None
        self.flags = torch.zeros(S, dtype=torch.int32, device=self.dev)
        tabs, keep = {}, []
        descs = (_lib.ChainDesc * S)()
        for s, b in enumerate(self.builts):
            key = (tuple(b["angle_h"].items()), tuple(b["angle_v"].items()))
            if key not in tabs:
                th, tv = _tables(b, n)
                tabs[key] = (torch.from_numpy(th).to(self.dev), torch.from_numpy(tv).to(self.dev))
            th, tv = tabs[key]
            d = descs[s]
            mir = G.mirrors_of(b)
            d.n_mirrors = K
            for k, m in enumerate(mir):
                d.negative[k] = int(m.negative)
                for c in range(10):
                    d.coeffs[k][c] = m.coeffs[c]
            d.dir = None
            d.tan_h, d.tan_v, d.n_h, d.n_v, d.ray0, d.n_rays = D.ptr(th), D.ptr(tv), n, n, 0, N
            d.org = None
            for c in range(3):
                d.src[c] = float(b["source"][c])
            d.last_hit, d.last_hit_ld = D.ptr(self.pt[s]), N
            d.dir_out, d.dir_out_ld = D.ptr(self.dir[s]), N
            if want_hits:
                d.hits, d.hits_ld = D.ptr(self.hits[s]), N
            d.samp_v_col = -1
            d.flags = D.ptr(self.flags[s:s + 1])
        self._tabs = tabs
        _lib.check(L.akb_trace_chain_batch_f64(descs, S, D.stream_handle()))
        flags = self.flags.cpu().numpy()
        for s in np.nonzero(flags)[0]:
            self._staged(int(s), tabs, n)
        self.s2f = np.array([b["s2f_middle"] for b in self.builts], dtype=np.float64)
        self.rot = self._rotations() if tilt else None

    def _staged(self, s, tabs, n):
        """The reference's stage-by-stage value rules for a flagged system (all-NaN on a miss)."""
        b = self.builts[s]
        key = (tuple(b["angle_h"].items()), tuple(b["angle_v"].items()))
        th, tv = tabs[key]
        from .trace import grid_dirs
        dirs = grid_dirs(th, tv)
        src = torch.tensor(b["source"], dtype=D.F64, device=self.dev).reshape(3, 1).expand(3, self.N).contiguous()
        hits, ray, _ = staged_chain(G.mirrors_of(b), dirs, src)
        self.dir[s].copy_(ray)
        self.pt[s].copy_(hits[-1])
        if self.hits is not None:
            for k, h in enumerate(hits):
                self.hits[s, k].copy_(h)

    def _rotations(self):
        """theta_y = -nanmean(arctan(angle[2]/angle[0])), theta_z = nanmean(arctan(angle[1]/angle[0]))
        (:3583-3588; np.mean in KB_debug, :11705-11706) and rotate_vectors' R_y(-theta_y),
        R_z(-theta_z) (:917-927), per system."""
        mean = np.nanmean if self.theta_mean == "nanmean" else np.mean
        ang = self.dir.cpu().numpy()
        rot = np.empty((self.S, 18), dtype=np.float64)
        self.thetas = np.empty((self.S, 2), dtype=np.float64)
        with np.errstate(invalid="ignore", divide="ignore"):
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)  # an all-NaN system: nanmean warns, gives NaN
                for s in range(self.S):
                    a = ang[s]
                    theta_y = -mean(np.arctan(a[2, :] / a[0, :]))
                    theta_z = mean(np.arctan(a[1, :] / a[0, :]))
                    self.thetas[s] = theta_y, theta_z
                    ry, rz = P.rotation_matrices(-theta_y, -theta_z)
                    rot[s, :9] = ry.ravel()
                    rot[s, 9:] = rz.ravel()
        self.theta = rot
        return torch.from_numpy(rot).to(self.dev)

    def evaluate(self, defocus, want_rows=False, systems=None):
        """np.std of the detector hits' z and y for each system against its planes
        x = s2f_middle + defocus[s][p] (coeffs_det[9] = -(s2f_middle + defocus), :2842-2845):
        (S, P) arrays size_v, size_h; with want_rows also the detcenter / angle rows (S, P, 3, N)."""
        L = _lib.lib()
        sel = list(range(self.S)) if systems is None else list(systems)
        dfc = np.asarray(defocus, dtype=np.float64)
        if dfc.ndim == 1:
            dfc = np.broadcast_to(dfc, (len(sel), dfc.shape[0]))
        Pn = dfc.shape[1]
        j = np.empty((len(sel), Pn), dtype=np.float64)
        for r, s in enumerate(sel):
            j[r] = -(self.s2f[s] + dfc[r])
        idx = torch.as_tensor(sel, device=self.dev)
        dirs = self.dir if systems is None else self.dir.index_select(0, idx).contiguous()
        pts = self.pt if systems is None else self.pt.index_select(0, idx).contiguous()
        rot = None
        if self.rot is not None:
            rot = self.rot if systems is None else self.rot.index_select(0, idx).contiguous()
        S = len(sel)
        jd = torch.from_numpy(j).to(self.dev)
        out = torch.empty((S, Pn, 2), dtype=D.F64, device=self.dev)
        det = ang = None
        if want_rows:
            det = torch.empty((S, Pn, 3, self.N), dtype=D.F64, device=self.dev)
            ang = torch.empty((S, Pn, 3, self.N), dtype=D.F64, device=self.dev)
        wb = int(L.akb_focus_eval_work_bytes(S, Pn, self.N))
        work = torch.empty(max(wb // 8, 1), dtype=D.F64, device=self.dev)
        _lib.check(L.akb_focus_eval_f64(D.ptr(dirs), D.ptr(pts), self.N, 3 * self.N, S, Pn, D.ptr(jd),
                                        D.ptr(rot) if rot is not None else None, D.ptr(out),
                                        D.ptr(det) if det is not None else None,
                                        D.ptr(ang) if ang is not None else None, D.ptr(work), D.stream_handle()))
        o = out.cpu().numpy()
        if want_rows:
            return o[..., 0], o[..., 1], det, ang
        return o[..., 0], o[..., 1]


def plot_result_test(params, source_shift=(0.0, 0.0, 0.0), option_tilt=True, *, option_set=True, ray_num=53,
                     as_torch=False):
    """plot_result_debug(params, 'test', source_shift=..., option_tilt=...) (:1326, 'test' mode):
    (vmirr_hyp, hmirr_hyp0, vmirr_ell, hmirr_ell, detcenter, angle) as numpy (3, 53^2) arrays, or
    np.inf where the reference returns np.inf."""
    b = G.build_akb(params, source_shift=source_shift, option_set=option_set)
    if not isinstance(b, dict):
        return b
    ts = TracedSystems([b], ray_num=ray_num, want_hits=True, tilt=option_tilt)
    _, _, det, ang = ts.evaluate(np.array([b["defocus"]]), want_rows=True)
    h = ts.hits[0]
    out = (h[0], h[3], h[1], h[2], det[0, 0], ang[0, 0])
    if as_torch:
        return out
    return tuple(x.cpu().numpy() for x in out)


def kb_test(params, source_shift=(0.0, 0.0, 0.0), *, designparams=None, ray_num=53, as_torch=False):
    """KB_debug(params, na_ratio_h, na_ratio_v, 'test') (:9742-12726; the NA ratios are unused):
    the KB pair of geometry.build_kb traced once, the detector hits tilted by the np.mean exit
    angles (always: the mode sets option_tilt = True, :11703-11717). Returns (vmirr_hyp, tilted
    hmirr_hyp, tilted detcenter, tilted angle) as numpy (3, n^2) arrays, or np.inf where the
    reference returns np.inf."""
    b = G.build_kb(params, source_shift=source_shift, designparams=designparams)
    if not isinstance(b, dict):
        return b
    ts = TracedSystems([b], ray_num=ray_num, want_hits=True, tilt=True, theta_mean="mean")
    _, _, det, ang = ts.evaluate(np.array([b["defocus"]]), want_rows=True)
    # the H hits rotated about the untilted spot's mean (:11708-11709), as rotate_points does
    det1 = np.array(b["det1"], dtype=np.float64)
    det0 = P.plane_ray_intersection(det1, ts.dir[0], ts.pt[0])
    focus = np.mean(det0.cpu().numpy(), axis=1)
    theta_y, theta_z = ts.thetas[0]
    h_rot = P.rotate_points(ts.hits[0, 1], focus, -theta_y, -theta_z)
    out = (ts.hits[0, 0], h_rot, det[0, 0], ang[0, 0])
    if as_torch:
        return out
    return tuple(x.cpu().numpy() for x in out)


class _SystemCache:
    """Built and traced systems keyed by what they depend on (params[1:], source shift, flags).
    system 'kb' builds KB_debug's pair (geometry.build_kb: no source shift - auto_focus_NA calls
    KB_debug without one - and always tilted by the np.mean angles)."""

    def __init__(self, option_set, ray_num, system="akb", kb_design=None):
        if system not in ("akb", "kb"):
            raise ValueError("system is 'akb' or 'kb'")
        self.option_set, self.ray_num, self.system = option_set, ray_num, system
        self.kb_design = kb_design
        self._c = {}

    def get(self, params, source_shift, tilt):
        kb = self.system == "kb"
        if kb:
            source_shift, tilt = (0.0, 0.0, 0.0), True
        key = (tuple(float(x) for x in np.asarray(params, dtype=np.float64)[1:]),
               tuple(float(x) for x in source_shift), bool(tilt))
        ts = self._c.get(key)
        if ts is None:
            if kb:
                b = G.build_kb(params, designparams=self.kb_design)
            else:
                b = G.build_akb(params, source_shift=source_shift, option_set=self.option_set)
            if not isinstance(b, dict):
                # the reference's plot_result_debug / KB_debug returns np.inf here and
                # auto_focus_NA's unpacking of it raises
                raise TypeError("cannot unpack non-iterable float object")
            ts = TracedSystems([b], ray_num=self.ray_num, tilt=tilt, theta_mean="mean" if kb else "nanmean")
            if len(self._c) > 64:
                self._c.clear()
            self._c[key] = ts
        return ts


def auto_focus_NA(num_adj_astg, initial_params, na_ratio_h, na_ratio_v, option, option_param, option_disp='ray',
                  option_mode=False, source_shift0=[0., 0., 0.], option_legendre=False, *, widesearch=False,
                  option_set=True, option_AKB=True, kb_design=None, driver=None, verbose=True, cache=None):
    """auto_focus_NA (AKB_raytrace_20250312.py:12746-12895) for the AKB system (option_AKB): the same
    ranges, steps, attempts, astigmatism updates and stopping rule, with every 100-value sweep of
    params[0] one device evaluation. initial_params is updated in place as the reference does.

    widesearch / option_set / option_AKB: the reference's module flags (:98, :94, :80). With
    option_AKB False the sweeps trace KB_debug's pair (kb_test's system: no source shift, always
    tilted by the np.mean angles, :12784; kb_design: the module's KBdesign_7params, :100).
    driver: the reference module, used only for what follows the search when `option` or
    `option_legendre` asks for a display or 'ray_wave' run (those call its own plot_result_debug /
    KB_debug; without a driver they raise)."""
    cache = cache or _SystemCache(option_set, 53, "akb" if option_AKB else "kb", kb_design)
    if widesearch:
        a_min, a_max = -1 + initial_params[0].copy(), 1 + initial_params[0].copy()
        shrink_factor, num_adj_astg, max_attempts = 0.1, 300, 17
    else:
        a_min, a_max = -0.3 + initial_params[0].copy(), 0.3 + initial_params[0].copy()
        shrink_factor, num_adj_astg, max_attempts = 0.1, 100, 16
    foc = option_mode == 'FoC'
    tilt = not foc

    def sweep(a):
        ts = cache.get(initial_params, source_shift0, tilt)
        size_v_, size_h_ = ts.evaluate(a)
        initial_params[0] = np.float64(a[-1])  # the reference's loop leaves the last value there
        return size_v_[0].copy(), size_h_[0].copy()

    attempt = 0
    a = best_a = axial_distance = size_v_param = size_h_param = None
    size_v_ = size_h_ = None
    while attempt < max_attempts:
        a = np.linspace(a_min, a_max, num_adj_astg)
        size_v_, size_h_ = sweep(a)
        if not foc:
            astig_shift = a[np.argmin(size_h_)] - a[np.argmin(size_v_)]
            initial_params[1] = initial_params[1] - astig_shift
        size_v_param = np.min(size_v_)
        size_h_param = np.min(size_h_)
        if not np.argmin(size_h_) == np.argmin(size_v_) and not foc:
            size_v_, size_h_ = sweep(a)
            astig_shift = a[np.argmin(size_h_)] - a[np.argmin(size_v_)]
            initial_params[1] = initial_params[1] - astig_shift
            size_v_param = np.min(size_v_)
            size_h_param = np.min(size_h_)
        initial_params[0] = a[np.argmin(size_h_)]
        best_a = initial_params[0]
        delta_a = (a_max - a_min) * shrink_factor
        a_min = best_a - delta_a / 2
        a_max = best_a + delta_a / 2
        distance_ = np.sqrt(size_v_**2 + size_h_**2)
        axial_distance = a[np.argmin(size_h_)] - a[np.argmin(size_v_)]
        if axial_distance <= 1e-11 and axial_distance > 1e-15:
            if verbose:
                print(f" attempt :{attempt}")
            break
        attempt += 1
    if verbose:
        print(f"  Optimal 'a': {best_a}, distance: {axial_distance}")
        print(f"  size_v_param: {size_v_param}, size_h_param: {size_h_param}\n")
        print(f"       v_shift: {a[np.argmin(size_v_)]},      h_shift: {a[np.argmin(size_h_)]}\n")
        print(f"  astigmatism: {initial_params[1]}")
        if attempt == max_attempts:
            print("Warning: Maximum attempts reached. Returning current best result.")
    if option_param == 'FoC':
        return plot_result_test(initial_params, source_shift0, option_tilt=False, option_set=option_set)[4]
    if option_legendre or option:
        if driver is None:
            raise NotImplementedError("the display / 'ray_wave' follow-up runs the reference's plot_result_debug: "
                                      "pass driver=<the AKB_raytrace module>")
        if option_legendre:
            if not option_AKB:
                return driver.KB_debug(initial_params, na_ratio_h, na_ratio_v, 'ray_wave', option_legendre=True,
                                       source_shift=source_shift0)
            return driver.plot_result_debug(initial_params, 'ray_wave', option_legendre=True, source_shift=source_shift0)
        if not option_AKB:
            r = driver.KB_debug(initial_params, na_ratio_h, na_ratio_v, option_disp)
            if option_disp == 'ray_wave':
                return r
        elif option_disp == 'ray_wave':
            return driver.plot_result_debug(initial_params, option_disp, source_shift=source_shift0)
        else:
            kw = dict(option_tilt=False) if foc else {}
            driver.plot_result_debug(initial_params, option_disp, source_shift=source_shift0, **kw)
    if option_param == 'D':
        return np.min(distance_)
    return size_v_param, size_h_param, initial_params


def calc_FoC(initial_params, range_h=[-5e-3, 5e-3, 15], range_v=[-5e-3, 5e-3, 15], *, option_set=True,
             verbose=False):
    """calc_FoC (:13766-13793) without its plots: for each source shift (0, h, v) on the grid, the
    FoC-mode auto_focus_NA (which carries params[0] from one source to the next, as the reference's
    in-place updates do) and the untilted spot's mean position and extent. Returns a dict of the
    (len(range_v), len(range_h)) arrays focuspointX/Y/Z, focussizeH/V."""
    range_h = np.linspace(range_h[0], range_h[1], range_h[2])
    range_v = np.linspace(range_v[0], range_v[1], range_v[2])
    shape = (len(range_v), len(range_h))
    out = {k: np.zeros(shape) for k in ("focuspointX", "focuspointY", "focuspointZ", "focussizeH", "focussizeV")}
    cache = _SystemCache(option_set, 53)
    for i in range(len(range_v)):
        for j in range(len(range_h)):
            S0 = [0., range_h[j], range_v[i]]
            det = auto_focus_NA(50, initial_params, 1, 1, True, 'FoC', option_mode='FoC', source_shift0=S0,
                                option_set=option_set, verbose=verbose, cache=cache)
            fp = np.mean(det, axis=1)
            out["focuspointX"][i, j], out["focuspointY"][i, j], out["focuspointZ"][i, j] = fp
            out["focussizeH"][i, j] = np.max(det[1, :]) - np.min(det[1, :])
            out["focussizeV"][i, j] = np.max(det[2, :]) - np.min(det[2, :])
    return out
