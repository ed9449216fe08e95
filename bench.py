"""Benchmark: ray-surface intersections/s of the 4-mirror AKB wavefront hot path (+ PSF wall time).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], "C3"): the 'ray_wave' path of plot_result_debug
(AKB_raytrace_20250312.py:1326) on a 3163 x 3163 ray grid (1.0e7 rays) per GPU through the
reference's Wolter III+I geometry (tests/golden/akb_geometry.json, recorded from the reference),
each step a different system of a cycle of --systems variants (the last mirror and the two
detector planes moved per system, as the focus sweeps move the system between traces):
pass 1 (4 mirrors), equal-angle resample, pass 2 (4 mirrors + OPL), tilt, two detector planes,
OPD; then a 128 x 128 pupil padded x16 -> 2048^2 PSF (pruned 2-D DFT: the padded plane is never
built). One step = all of it; its intersections are 2 passes x 4 mirrors x rays. Steps are
pipelined the way a caller tracing many systems would run them (RayWave.launch_front /
launch_back): by default (--fuse 2) step k's pass-1 kernel also tilts step k-2 and forms step
k-3's OPD maps (their loads hidden behind the chain's FP64 arithmetic), step k-1's pass-2 sums and
tilt parameters finish on their own stream beside step k's passes, and step k-3's pupil and PSF
run on other streams beside step k's pass 2 while the host resamples. Every step still does
all of its work inside the timed region. Inputs (the two 1-D angle tables) are resident on the
device before timing.

--config c2 (configs[1]): the same pipeline through KB_debug's pair at params = 0
(geometry.build_kb, bit-exact vs the reference's builds; the second plane at the module's
defocusForWave = 1e-3, :89, as its 'wave' mode places it, :11694-11698): 2 passes x 2 mirrors per
ray; huygens_pairs_per_s is that config's M2 -> image stage.

Multi-GPU (configs[3], "C4"): weak scaling at C4's per-GPU load, ~1.25e7 rays per rank of a
round(sqrt(N * 1.25e7))^2 grid - 10000^2 = 1e8 rays, ~1250 V-rows per rank, at N = 8 - in
contiguous blocks of whole 8192-ray numpy sum buffers (Shard.split), so the cross-rank means are
numpy's to the bit; the exchanges are tiny all-gathers / all-reduces and the pupil before the PSF
on rank 0.

Prints one JSON line (rank 0). The dominant kernel's roofline uses HIP events on the stream it runs
on; its PMC-derived fields (HBM traffic, FP64 rate, the VALU-issue roofline) come from the newest
profiles/*_roofline.json whose source hash matches the trace kernels' sources, else null.
cpu_baseline times the oracle's C restatement (the "port") on this host on a bounded sample.
Outside the timed region: one run() with its host wait (single_run_ms); at N = 1 also the
faithful PSF chain (griddata + plane correction + psf_calc, faithful_psf_chain_ms) and the
Huygens stage of configs[1] (huygens_pairs_per_s).
"""
import argparse
import ctypes
import glob
import json
import math
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ray-surface intersections/sec + PSF wall-time, 1e7-ray 4-mirror AKB, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md
FP64_VALU_PEAK_TFS = 78.6  # MI355X FP64 vector peak (FMA counted as 2 flops)
SIMDS = 1024  # 256 CUs x 4 SIMDs; a wave64 VALU instruction occupies a SIMD for 4 cycles
C3_RAYS = 1.0e7  # configs[2]: 1e7 rays on one GPU
C4_RAYS_PER_GPU = 1.25e7  # configs[3]: 1e8 rays over 8 GPUs
# bytes the pass-2 chain kernel must move per ray: it reads two L2-resident 1-D tables and
# writes last hit (24) + exit direction (24) + OPL (8); the arctans and detector hits it also
# forms are reduced in-kernel (numpy-order leaf sums, 5 x 8 B per 128 rays)
PASS2_BYTES_PER_RAY = 56


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # the device's clock settles over the first ~25 steps of a fresh process (step lengths fall
    # from ~1.0 to ~0.8 ms, scripts/step_timeline.py): the default warm-up covers that
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=30, help="at least 3 with --fuse 2 (fills the pipeline)")
    # a fresh process's device clock settles over ~0.3 s of load: the driver's 20 steps after 5
    # warm-up steps measured 0.89 ms per step without a ramp, 0.80 with it (100 / 30: 0.78);
    # the timed steps are the same either way, and the JSON line reports the ramp
    p.add_argument("--ramp-ms", type=float, default=300.0,
                   help="device clock ramp before the warm-up: untimed steps for this long (reported)")
    p.add_argument("--rays", type=float, default=None,
                   help="rays per GPU (default: 1e7 on one GPU, C3; 1.25e7 per rank at N > 1, C4's 1e8 at N = 8)")
    p.add_argument("--systems", type=int, default=8,
                   help="distinct systems cycled through the steps (1: the same system every step)")
    p.add_argument("--no-extras", action="store_true",
                   help="skip single_run_ms / faithful_psf_chain_ms / huygens_pairs_per_s")
    p.add_argument("--pupil", type=int, default=128)
    p.add_argument("--faithful-steps", type=int, default=10,
                   help="steps of the trace + faithful-PSF loop reported as faithful_step (outside the timed region)")
    p.add_argument("--pad", type=int, default=16)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--config", choices=("c2", "c3", "c5"), default="c3",
                   help="c3: BASELINE configs[2] (default, the headline); c5: configs[4], the Legendre "
                        "figure-error OPL perturbation on every ray + a 3-wavelength PSF stack; c2: configs[1], "
                        "the KB pair")
    p.add_argument("--back-stream", type=int, default=1,
                   help="1: queue each step's tilt / OPD / pupil on a second stream, concurrent with the "
                        "next step's FP64-bound pass 1 (0: behind it on one stream)")
    p.add_argument("--back-priority", type=int, default=0,
                   help="torch stream priority of the back stream (lower = higher priority; 0 = normal)")
    p.add_argument("--reserve-cus", type=int, default=None,
                   help="CUs (a multiple of 8 up to 128, the same number on every XCD) the main stream's passes leave "
                        "to the other streams (akb_stream_create_reserved), where the faithful chain's "
                        "single-workgroup kernels then start without waiting for a CU to drain (default 40 at "
                        "N = 1, measured best of 0..96; 0 at N > 1, unmeasured there)")
    p.add_argument("--fuse", type=int, default=2,
                   help="2: step k's pass-1 kernel also tilts step k-2 and forms step k-3's OPD maps (their loads "
                        "hidden behind the chain's FP64 arithmetic), step k-3's pupil / PSF on the back stream; "
                        "1: the tilt only, the OPD on the back stream; 0: the tilt as its own kernel on the back "
                        "stream beside pass 1")
    p.add_argument("--pupil-mode", choices=("faithful", "standin"), default="faithful",
                   help="faithful (default): each step's PSF is the reference's own - griddata(cubic) of Wave2 "
                        "(cone solve), nanmean removal, plane correction, psf_calc - pipelined on the back stream "
                        "(akbraytracing_amd/faithful.py); standin: RayWave.pupil's ray-index sampler (rounds 1-3)")
    p.add_argument("--cone-sweeps", type=int, default=None,
                   help="Chebyshev sweeps of the faithful pupil's cone solve (default griddata.CONE_SWEEPS)")
    p.add_argument("--begin-stream", choices=("back", "fin", "copy"), default="back",
                   help="stream of the faithful pupil's begin (cell pass + ring copy): the back stream, or "
                        "RayWave's finish / copy stream (N = 1), waiting for the run's back half")
    p.add_argument("--faithful-lag", type=int, default=None,
                   help="faithful runs in flight (begun, not finished) after each step: the oldest finishes once "
                        "more are (default 3; 6 at N > 1, where the band owner builds configs[3]'s 40k-point ring)")
    p.add_argument("--step-log", action="store_true",
                   help="add step_log to the line: per timed step, when its main-stream and back-stream work "
                        "completed (ms after the region's start, device events) and its host time / wait")
    p.add_argument("--no-ramp-form", action="store_true",
                   help="skip the timed steps before the clock ramp (ms_per_step_no_ramp)")
    p.add_argument("--psf-start", choices=("pupil", "pass1"), default="pupil",
                   help="side-stream PSF starts as soon as the previous pupil is ready, beside pass 1 "
                        "(default; measured faster), or after this step's pass 1")
    return p.parse_args()


def workload_label(config, world, faithful):
    """config.workload: the configuration, what a step runs, and the pupil route"""
    pupil = (" + the reference's pupil (griddata cubic, nanmean, plane correction, psf_calc)"
             + (" sharded with the rays" if world > 1 else "")) if faithful else ""
    shards = ", ray-row shards" if world > 1 else ""
    if config == "c2":
        return f"C2: 2-mirror KB ray trace (2 passes, tilt, OPD){shards}{pupil} + 2048^2 PSF"
    if config == "c3":
        name = "C3" if world == 1 else "C4"
        return f"{name}: 4-mirror AKB ray_wave trace (2 passes, tilt, OPD){shards}{pupil} + 2048^2 PSF"
    return ("C5: 4-mirror AKB ray_wave trace with per-ray Legendre OPL perturbation" + shards + pupil
            + " + 3-wavelength 2048^2 PSF stack")


def geometry_dict(config):
    """The traced system as a dict: the recorded AKB fixture (c3, c5) or KB_debug's pair built
    from params = 0 with its 'wave'-mode second plane (c2)."""
    if config != "c2":
        with open(os.path.join(ROOT, "tests", "golden", "akb_geometry.json")) as f:
            return json.load(f)
    import numpy as np
    from akbraytracing_amd import geometry as G
    b = G.build_kb(np.zeros(26))
    det2 = np.zeros(10)
    det2[6] = 1
    det2[9] = -(np.float64(b["s2f_middle"]) + np.float64(b["defocus"]) + 1e-3)
    return dict(b, det2=[float(x) for x in det2], defocus_wave_m=1e-3)


def cpu_baseline(seconds, g):
    """The oracle (C restatement, OpenMP, + numpy for the host steps) running the same ray_wave
    pipeline on a 1001^2 grid, repeated for about `seconds`."""
    import oracle
    import oracle.pipeline as OPL
    threads = oracle.max_threads()
    n = 1001
    OPL.akb_ray_wave(g, 65)  # load / warm
    reps, t0 = 0, time.perf_counter()
    while True:
        OPL.akb_ray_wave(g, n)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 1000:
            break
    inter = 2 * len(g["mirrors"]) * n * n * reps
    # the same pipeline on one thread (SURVEY.md §8(d) asks for both), a shorter sample
    oracle.set_threads(1)
    n1, reps1, t1 = 501, 0, time.perf_counter()
    try:
        while True:
            OPL.akb_ray_wave(g, n1)
            reps1 += 1
            el1 = time.perf_counter() - t1
            if el1 >= seconds / 4 or reps1 >= 1000:
                break
    finally:
        oracle.set_threads(threads)
    one = 2 * len(g["mirrors"]) * n1 * n1 * reps1 / el1
    return {"value": inter / el, "unit": "intersections/s", "cores": threads, "kind": "port",
            "sample": f"oracle ray_wave pipeline (C primitives, OpenMP {threads} threads, numpy means/interp1d) "
                      f"on a {n}x{n} grid, {reps} reps in {el:.1f} s",
            "value_1thread": one,
            "sample_1thread": f"same pipeline, 1 thread, {n1}x{n1} grid, {reps1} reps in {el1:.1f} s"}


def _tag_key(path):
    """Order of profile tags: rNN then the run letters a .. z, aa .. zz (so r05y < r05aa)."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def _pick_profile(files, sha):
    """(summary, file, matches) of the newest of files whose sources_sha256 is sha, else of the
    newest one."""
    files = sorted(files, key=_tag_key, reverse=True)
    if not files:
        return {}, None, False
    docs = []
    for f in files:
        with open(f) as fh:
            docs.append(json.load(fh))
        if docs[-1].get("sources_sha256") == sha:
            return docs[-1], os.path.relpath(f, ROOT), True
    return docs[0], os.path.relpath(files[0], ROOT), False


def read_profile():
    """(summary, file, matches): the newest profiles/*_roofline.json (scripts/summarize_profiles.py)
    that describes these kernel sources (its sha256 of them equals theirs now), else the newest."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from summarize_profiles import sources_sha256
    files = [f for f in glob.glob(os.path.join(ROOT, "profiles", "*_roofline.json"))
             if not f.endswith("_faithful_roofline.json")]
    return _pick_profile(files, sources_sha256())


def system_variants(geom, k):
    """k distinct systems on geom's ray grid: the last mirror's constant term scaled by
    1 + 2e-11 i and the two detector planes moved 3 and 5 um x i (i = 0 .. k-1)."""
    import copy
    out = []
    for i in range(k):
        g = copy.deepcopy(geom)
        c = list(g.mirrors[-1].coeffs)
        c[9] = c[9] * (1.0 + 2e-11 * i)
        g.mirrors[-1].coeffs = c
        g.det1 = list(g.det1[:3]) + [g.det1[3] - 3e-6 * i]
        if g.det2 is not None:
            g.det2 = list(g.det2[:3]) + [g.det2[3] - 5e-6 * i]
        out.append(g)
    return out


def faithful_psf(out, n, size):
    """The reference's own PSF of one trace: griddata(cubic) of Wave2 from the
    detector-2 hits onto a size x size grid, nanmean removal, plane correction (pupilmap.wave_pupil),
    then psf_calc (rotation estimate, rotate_with_nan, pad-16 PSF, trim)."""
    from akbraytracing_amd import pupilmap as PM
    from akbraytracing_amd.psfcalc import psf_calc
    m, gh, gv, _ = PM.wave_pupil(out["detcenter2"], out["wave2"], n, n, grid_num_H=size, grid_num_V=size)
    return psf_calc(m, gh, gv, 1e-2)


def faithful_psf_chain(rw, out, size, reps=5):
    """Wall time (ms, device synchronised, host steps included; median of reps) of faithful_psf on
    the last step's trace, and of the driver's whole gridding step (pupilmap.wave_maps: DistError2's
    map too, which feeds no PSF) + psf_calc."""
    import torch
    from akbraytracing_amd import pupilmap as PM
    from akbraytracing_amd.psfcalc import psf_calc
    det2 = out["detcenter2"].clone()
    e2, w2 = out["dist_err2"].clone(), out["wave2"].clone()
    src = dict(detcenter2=det2, wave2=w2)

    def timed(f):
        times = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        return sorted(times)[reps // 2]

    def both():
        m = PM.wave_maps(det2, e2, w2, rw.n, rw.n, grid_num_H=size, grid_num_V=size)
        psf_calc(m["matrixWave2_Corrected"], m["grid_H"], m["grid_V"], 1e-2)

    return timed(lambda: faithful_psf(src, rw.n, size)), timed(both)


def huygens_rate(out):
    """configs[1]'s M2 -> image stage shape: this run's last-mirror hits as
    sources (unit field, dS = 1) onto a 65 x 65 image grid around the focus; pairs/s."""
    import numpy as np
    import torch
    from akbraytracing_amd.wavecalc import propagate
    src = out["last_hit"]
    sx, sy, sz = (src[i].contiguous() for i in range(3))
    u = torch.ones(sx.shape[0], dtype=torch.complex128, device=sx.device)
    c = out["detcenter2"].mean(dim=1).cpu().numpy()
    t = np.linspace(-1e-6, 1e-6, 65)
    ty, tz = np.meshgrid(c[1] + t, c[2] + t)
    T = [torch.from_numpy(np.ascontiguousarray(v.ravel())).to(sx.device) for v in (np.full(ty.size, c[0]), ty, tz)]
    k = 2 * np.pi / 13.5e-9
    propagate(*T, sx, sy, sz, u, k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        propagate(*T, sx, sy, sz, u, k)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 3
    rate = T[0].shape[0] * sx.shape[0] / (ms * 1e-3)
    res = {"value": rate, "unit": "pairs/s", "ms": ms, "sources": int(sx.shape[0]), "targets": int(T[0].shape[0]),
           "stage": "M2 -> 65x65 image grid (configs[1]'s stage shape, sources from this trace)"}
    # its roofline: VALU issue (FP64 sqrt / reciprocal / sincos per pair, sources from LDS) with the
    # instruction mix of the committed PMC summary (scripts/summarize_huygens.py) while it describes
    # this kernel source
    import hashlib
    src = os.path.join(ROOT, "akbraytracing_amd", "csrc", "akb_huygens.hip")
    prof, pfile, ok = _pick_profile(glob.glob(os.path.join(ROOT, "profiles", "*_huygens.json")),
                                    hashlib.sha256(open(src, "rb").read()).hexdigest())
    if ok:
        lane_ops = prof["valu_lane_ops_per_pair"]
        peak = SIMDS / 4 * prof["effective_clock_ghz"] * 1e9 * 64 / lane_ops
        res["roofline"] = {"bound": "valu-issue", "achieved": rate, "peak": peak, "unit": "pairs/s",
                           "frac": rate / peak, "valu_lane_ops_per_pair": lane_ops,
                           "fp64_lane_ops_per_pair": prof["fp64_lane_ops_per_pair"],
                           "non_fp64_share": prof["non_fp64_share"],
                           "fp64_frac_of_peak_profiled": prof["fp64_frac_of_peak"],
                           "issue_frac_profiled": prof["issue_frac"],
                           "effective_clock_ghz": prof["effective_clock_ghz"]}
    res["profile"] = {"file": pfile, "matches_sources": ok}
    return res


def read_faithful_profile():
    """(summary, file, matches): the newest profiles/*_faithful_roofline.json (scripts/
    summarize_profiles.py: PMC of the cone solve's kernels) that describes these sources, else the
    newest."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from summarize_profiles import GD_SOURCES, sources_sha256
    return _pick_profile(glob.glob(os.path.join(ROOT, "profiles", "*_faithful_roofline.json")),
                         sources_sha256(sources=GD_SOURCES))


def faithful_roofline(ms, cells, K, S):
    """The cone solve's patch kernel (k_gd_cone_patch) over the timed steps: its launch time from HIP
    events around every launch (akb_gd_patch_times, in the step, sharing the GPU), its work (interior
    target cells x the box's shrinking squares: sum_j (2K + 4 - 2j)^2 vertex-sweeps; (W - 2)^2 vertex
    setups, each vertex's constants formed once per cell), its compulsory HBM traffic (the cells' boxes
    of x, y, f and diagonal bytes in, four corners' gradients out) against 8 TB/s, and - from the
    committed PMC summary while it describes these sources - its VALU issue against the SIMDs'."""
    W = 2 * K + 4
    sweeps = sum((W - 2 * j) ** 2 for j in range(1, K + 1))
    setups = (W - 2) ** 2
    avg = sum(ms) / len(ms)
    byts = cells * (W * W * 24 + (W - 1) * (W - 1) + 4 * 16)
    prof, pfile, pok = read_faithful_profile()
    pk = prof.get("kernels", {}).get("cone_patch", {}) if pok else {}
    valu = pk.get("valu_wave_instructions_per_launch")
    clock = pk.get("effective_clock_ghz")
    out = {
        "kernel": "k_gd_cone_patch (akb_griddata.hip)",
        "bound": "latency: one workgroup of (W-2)^2 + (W-2S-2)^2 vertex threads per CU, a barrier per sweep "
                 "(VALU issue below)",
        "launches": len(ms),
        "avg_ms": avg,
        "cells_per_launch": cells,
        "vertex_sweeps_per_launch": cells * sweeps,
        "vertex_setups_per_launch": cells * setups,
        "vertex_sweeps_per_s": cells * sweeps / (avg * 1e-3),
        "hbm": {"algorithmic_bytes_per_launch": byts, "achieved": byts / (avg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "traffic": pk.get("hbm_bytes_per_launch")},
        "valu_issue": {"wave_instructions_per_launch": valu, "effective_clock_ghz": clock,
                       "achieved": valu / (avg * 1e-3) if valu else None,
                       "peak": SIMDS / 4 * clock * 1e9 if clock else None, "unit": "wave-instructions/s",
                       "frac": (valu / (avg * 1e-3)) / (SIMDS / 4 * clock * 1e9) if valu and clock else None,
                       "lane_ops_per_vertex_sweep": 64 * valu / (cells * (sweeps + setups)) if valu and cells else None,
                       "lds_wave_instructions_per_launch": pk.get("lds_wave_instructions_per_launch"),
                       "lds_bank_conflict_cycles_per_launch": pk.get("lds_bank_conflict_cycles_per_launch"),
                       "wait_any_frac_profiled": pk.get("wait_any_frac"),
                       "issue_frac_profiled": pk.get("issue_frac")},
        "profile": {"file": pfile, "matches_sources": pok},
    }
    return out


# bytes pass 1 moves per ray besides its 2n-entry tables: the fused tilt of run k-2 reads the last
# hit and exit direction (48) + total OPL (8) and writes detector-2 hit (24) + total OPL 2 (8); the
# fused OPD of run k-3 reads t2 + detector-2 hit (32) and writes DistError2 and Wave2 (16)
PASS1_TILT_BYTES_PER_RAY = 88
PASS1_OPD_BYTES_PER_RAY = 48


def pass1_roofline(launches, rays, prof, fuse):
    """The pass-1 kernel of the timed steps: HIP-event time per launch (the steady-state launches:
    tilt and OPD fused when --fuse 2), its algorithmic bytes against 8 TB/s, and - from the committed
    PMC summary (its pass1_fused entry) while it describes these sources - its HBM traffic, VALU issue
    and wait fractions. Pass 1 is VALU-issue bound (4 mirrors of FP64 quadric solves per ray); its
    HBM bytes are the fused tilt / OPD rows it carries."""
    if not launches:
        return None
    full = [ms for ms, ft, fo in launches if ft and fo] if fuse >= 2 else \
           [ms for ms, ft, fo in launches if ft] if fuse == 1 else [ms for ms, _, _ in launches]
    ms = full or [ms for ms, _, _ in launches]
    avg = sum(ms) / len(ms)
    per_ray = (PASS1_TILT_BYTES_PER_RAY if fuse >= 1 else 0) + (PASS1_OPD_BYTES_PER_RAY if fuse >= 2 else 0)
    byts = per_ray * rays
    pk = prof.get("kernels", {}).get("pass1_fused", {}) if fuse >= 2 else {}
    clock = pk.get("effective_clock_ghz")
    valu = pk.get("valu_wave_instructions_per_launch")
    return {
        "kernel": "k_chain_tilt<4,true> (pass 1 + tilt of run k-2 + OPD of run k-3)" if fuse >= 2 else
                  "k_chain_tilt<4,false> (pass 1 + tilt of run k-2)" if fuse == 1 else "k_chain (pass 1, flags only)",
        "launches": len(ms),
        "avg_ms": avg,
        "rays_per_launch": rays,
        "hbm": {"bound": "hbm", "algorithmic_bytes_per_launch": byts,
                "achieved": byts / (avg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": pk.get("hbm_bytes_per_launch")},
        "valu_issue": {"bound": "valu-issue", "wave_instructions_per_launch": valu, "effective_clock_ghz": clock,
                       "achieved": valu / (avg * 1e-3) if valu else None,
                       "peak": SIMDS / 4 * clock * 1e9 if clock else None, "unit": "wave-instructions/s",
                       "frac": (valu / (avg * 1e-3)) / (SIMDS / 4 * clock * 1e9) if valu and clock else None,
                       "issue_frac_profiled": pk.get("issue_frac"), "wait_any_frac_profiled": pk.get("wait_any_frac"),
                       "non_fp64_share": pk.get("non_fp64_share")},
        "fusion_ab": "--fuse 2 / 1 / 0 (this kernel fused with tilt + OPD / tilt only / neither): 1.63 / 1.66 / "
                     "1.83 ms per step, two interleaved rounds (profiles/r06a_fuse_ab.json)",
    }


def rank0_tail(n=10000, reps=3, size=128, pad=16, lams=(13.5e-9,), workers=4):
    """C4's band owner's extra work per run, measured on one GPU. At N > 1 every rank
    traces its rows and forms the interior targets of its own cells (faithful_dist.py); rank 0 alone
    also iterates the boundary band (K + 1 launches), builds the pockets on the host (worker threads),
    and runs the post and the PSF. Here the one-process chain runs on configs[3]'s whole n^2 = 1e8-ray
    lattice (one trace of the C3 system) and its device phases are timed with HIP events: the band
    iteration (akb_gd_band_times), the post, the PSF, and the finish as a whole (with every interior
    patch: finish - patches bounds rank 0's device share from above); the pocket job's host time
    comes from its worker. Medians over reps runs after one first-use run."""
    import torch
    from akbraytracing_amd import _lib as LIBM
    from akbraytracing_amd.faithful import FaithfulPupil
    from akbraytracing_amd.wavefront import RayWave, SystemGeometry
    L = LIBM.lib()
    rw = RayWave(SystemGeometry.from_dict(geometry_dict("c3")), n)
    out = rw.run()
    d2, w2 = out["detcenter2"], out["wave2"]
    fp = FaithfulPupil(n, n, size=size, pad=pad, wavelengths=list(lams), slots=2, workers=workers)

    def ev():
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    rows = []
    try:
        for i in range(reps + 1):
            if i == 1:
                LIBM.check(L.akb_gd_patch_timing(1))
            e_fin, e_psf, e_post = ev(), ev(), ev()
            t = fp.begin(d2[1], d2[2], w2)
            fp.finish(t, events=e_fin, psf_events=e_psf, post_events=e_post)
            t.check()
            torch.cuda.synchronize()
            if i >= 1:
                rows.append({"finish": e_fin[0].elapsed_time(e_fin[1]), "psf": e_psf[0].elapsed_time(e_psf[1]),
                             "post": e_post[0].elapsed_time(e_post[1])})
        LIBM.check(L.akb_gd_patch_timing(0))
        bms = (ctypes.c_float * 64)()
        nb = L.akb_gd_band_times(bms, 64)
        pms = (ctypes.c_float * 64)()
        npch = L.akb_gd_patch_times(pms, None, 64)
        if nb < 0 or npch < 0:
            LIBM.check(min(nb, npch))
        pockets = list(fp.pocket_ms[1:])
    finally:
        fp.close()
    del rw, out, d2, w2, fp
    torch.cuda.empty_cache()

    def med(v):
        v = sorted(v)
        return v[len(v) // 2] if v else None

    band, patch = med(list(bms[:nb])), med(list(pms[:npch]))
    post, psf, fin = med([r["post"] for r in rows]), med([r["psf"] for r in rows]), med([r["finish"] for r in rows])
    return {"lattice": f"{n}^2 (configs[3]'s 1e8 rays, one GPU)", "runs": len(rows),
            "rank0_tail_ms": band + post + psf,
            "band_iteration_ms": band, "post_ms": post, "psf_ms": psf,
            "finish_ms": fin, "patches_ms": patch, "finish_minus_patches_ms": fin - patch,
            "pocket_job_host_ms": med(pockets), "pocket_workers": workers,
            "what": "rank0_tail_ms = the band owner's device-only work per run (band iteration + post + PSF), "
                    "alone on the GPU; finish_minus_patches_ms also holds the claims and the evaluation every "
                    "rank shares; the pocket job runs on the host beside the passes (pocket_job_host_ms / "
                    "pocket_workers per run of throughput)"}


def stage_api(rw, geom, dev, reps=5):
    """The drop-in stage API (SURVEY.md §8(d)'s HBM-bound mode): the reference's per-mirror calls
    on device-resident (3, N) rows of the bench's grid - mirr_ray_intersection, the segment norm,
    norm_vector, reflect_ray per mirror, then plane_ray_intersection (AKB_raytrace_20250312.py:
    2881-2905) - through the C ABI, each kernel timed over `reps` back-to-back calls with HIP events
    on the current stream. Algorithmic bytes per ray: the rows a call reads and writes."""
    import torch
    from akbraytracing_amd import _lib
    from akbraytracing_amd import device as D
    L = _lib.lib()
    n = rw.n * rw.n
    th, tv = rw.tan_h, rw.tan_v
    ih = torch.arange(n, device=dev) % rw.n
    iv = torch.arange(n, device=dev) // rw.n
    raw = torch.stack([torch.ones(n, dtype=torch.float64, device=dev), th[ih], tv[iv]]).contiguous()
    del ih, iv
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    sh = D.stream_handle()
    P = D.ptr

    def cf(c):
        return (ctypes.c_double * 10)(*[float(x) for x in c])

    def plane4(p):
        return (ctypes.c_double * 4)(*[float(x) for x in p])

    def timed(fn):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / reps

    res = {}
    d = torch.empty_like(raw)
    res["normalize_vector"] = (timed(lambda: _lib.check(L.akb_normalize_f64(P(raw), n, 1, n, P(d), n, P(flags), sh))), 48)
    o = torch.zeros_like(raw)  # the point source, as (3, N) rows
    hit = torch.empty_like(raw)
    nrm = torch.empty_like(raw)
    d2 = torch.empty_like(raw)
    seg = torch.empty(n, dtype=torch.float64, device=dev)
    per = {"mirr_ray_intersection": [], "segment_length": [], "norm_vector": [], "reflect_ray": []}
    torch.cuda.synchronize()
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    chain_ms = 0.0
    for m in geom.mirrors:
        q = cf(m.coeffs)
        neg = int(bool(m.negative))
        calls = [
            ("mirr_ray_intersection", lambda: _lib.check(L.akb_isect_f64(q, P(d), n, 1, P(o), n, 1, neg, n, P(hit), n, P(flags), sh))),
            ("segment_length", lambda: _lib.check(L.akb_seglen_f64(P(o), n, 1, P(hit), n, 1, n, P(seg), sh))),
            ("norm_vector", lambda: _lib.check(L.akb_normal_f64(q, P(hit), n, 1, n, P(nrm), n, 1, P(flags), sh))),
            ("reflect_ray", lambda: _lib.check(L.akb_reflect_f64(P(d), n, 1, P(nrm), n, 1, n, P(d2), n, 1, P(flags), sh))),
        ]
        c0.record()
        for _, fn in calls:  # the mirror once, in the reference's order (the chain's own time)
            fn()
        c1.record()
        c1.synchronize()
        chain_ms += c0.elapsed_time(c1)
        for name, fn in calls:
            per[name].append(timed(fn))
        d, d2 = d2, d
        o, hit = hit, o
    pl = plane4(geom.det2 or geom.det1)
    res["plane_ray_intersection"] = (timed(lambda: _lib.check(L.akb_plane_isect_f64(pl, P(d), n, 1, P(o), n, 1, n, P(hit), n, sh))), 72)
    nbytes = {"mirr_ray_intersection": 72, "segment_length": 56, "norm_vector": 48, "reflect_ray": 72}
    for k, v in per.items():
        res[k] = (sum(v) / len(v), nbytes[k])
    out = {}
    for k, (ms, b) in res.items():
        gbs = b * n / (ms * 1e-3) / 1e9
        out[k] = {"ms": ms, "bytes_per_ray": b, "gbs": gbs, "frac_of_hbm": gbs / 8000.0}
    k = len(geom.mirrors)
    out["chain"] = {"ms": chain_ms, "rays": n, "mirrors": k,
                    "intersections_per_s": k * n / (chain_ms * 1e-3),
                    "bytes_per_intersection": 248,
                    "gbs": 248 * k * n / (chain_ms * 1e-3) / 1e9,
                    "what": "per mirror: intersection, segment norm, normal, reflection as separate calls"}
    out["rays"] = n
    # the device's streaming ceiling for the same traffic: a (3, N) float64 copy (48 B per ray)
    cms = timed(lambda: d2.copy_(d))
    out["copy_3xN_f64"] = {"ms": cms, "gbs": 48 * n / (cms * 1e-3) / 1e9}
    return out


def _lib_hash():
    from akbraytracing_amd import _lib
    return _lib.sources_hash()


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run on 127.0.0.1 and return its exit code. Called before anything touches the
    GPU, so this process never initialises HIP (the ranks are its children, not an exec)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    args.warmup = max(args.warmup, 3 if args.fuse >= 2 else 1)
    import torch
    from akbraytracing_amd import build as B
    from akbraytracing_amd import dist as AD
    rank, world, local = AD.init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    if not os.path.exists(B.SO):
        if rank == 0:
            B.build()
        AD.TorchComm().barrier()
    from akbraytracing_amd.psf import psf_stack
    from akbraytracing_amd.wavefront import RayWave, Shard, SystemGeometry

    dev = torch.device("cuda", torch.cuda.current_device())
    if args.reserve_cus is None:
        args.reserve_cus = 40 if world == 1 else 0
    if args.reserve_cus:
        from akbraytracing_amd.device import reserved_stream
        torch.cuda.set_stream(reserved_stream(args.reserve_cus, dev))
    gdict = geometry_dict(args.config)
    geom = SystemGeometry.from_dict(gdict)
    if args.rays is None:
        args.rays = C3_RAYS if world == 1 else C4_RAYS_PER_GPU
    # 3163 at 1 GPU (C3); 10000 at 8 GPUs (C4: 1250 V-rows per rank); SURVEY.md §8(d)
    n = int(round(math.sqrt(args.rays * world))) if world > 1 else int(math.ceil(math.sqrt(args.rays)))
    systems = system_variants(geom, max(args.systems, 1))
    shard = Shard.split(n, world, rank)
    comm = AD.TorchComm(dev)
    pert = None
    lams = [13.5e-9]  # EUV, AKB_raytrace_20250312.py:1161-1162 / :3614
    if args.config == "c5":
        from akbraytracing_amd.legendre import LegendrePerturbation, config5_coefficients
        pert = LegendrePerturbation(config5_coefficients(lams[0]))
        lams = [13.5e-9, 1.35e-9, 1.35e-10]  # EUV, softXray, hardXray (:1161-1166)
    rw = RayWave(geom, n, shard=shard, comm=comm, perturbation=pert)
    nsteps = [0]  # steps launched so far (which system the next one traces)

    def sys_of(i):
        return systems[i % len(systems)]

    psf_events = []
    psf_out = {}
    # one stream for the back halves, pupils and PSFs (RayWave holds two more: with the caller's,
    # four streams on the box's four hardware queues per process, none shared)
    # --back-priority -1 lets the HBM-bound back half take CU slots ahead of the FP64-bound pass 1
    # it overlaps; measured a wash (the host resample then lands on the critical path), so off
    back_stream = torch.cuda.Stream(device=dev, priority=args.back_priority)
    state = {"psf_done": None}
    fronts = []  # launched fronts (pass 1 .. tilt parameters) whose back half is still to queue

    # the PSF stack is wavelength-sharded: rank r transforms lams[r::world]
    my_lams = AD.wavelength_shard(lams, world, rank)

    def run_psf(opd, pitch, ready, timed):
        """The PSF of a finished pupil on the back stream, right behind it: it shares the GPU with
        the next kernels of the main stream."""
        if not my_lams:
            return
        side = back_stream
        side.wait_event(ready)
        if args.psf_start == "pass1":
            after = torch.cuda.Event()
            after.record()
            side.wait_event(after)
        with torch.cuda.stream(side):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
            psf, _, _ = psf_stack(opd, None, my_lams, None, pitch=pitch, pad_factor=args.pad,
                                  out=psf_out.get("psf"))
            psf_out["psf"] = psf
            if timed:
                e1.record(side)
                psf_events.append((e0, e1))
            done = torch.cuda.Event()
            done.record(side)
        state["psf_done"] = done

    faithful = args.pupil_mode == "faithful"
    if args.faithful_lag is None:
        args.faithful_lag = 3 if world == 1 else 6
    fp = None
    tickets = []
    finished = []  # finished runs' tickets whose error words are still to be checked
    checked = {"runs": 0, "guard_trips": 0}

    def check_finished(block):
        """Each finished run's own error words (the reference's raises): those whose device work is
        done (block False: never waits - the timed steps' form), or all of them (block True). A cone
        guard trip (the cone solve's estimate over its bar: FaithfulPupil.run would re-form that map
        from the converged gradients) is counted, not raised; any other error raises."""
        from akbraytracing_amd.griddata import ConeNotConverged
        while finished and (block or finished[0].done is None or finished[0].done.query()):
            t = finished.pop(0)
            try:
                fp.check(t) if world > 1 else t.check()
            except ConeNotConverged:
                checked["guard_trips"] += 1
            checked["runs"] += 1

    fp_events = []
    if faithful and world == 1:
        from akbraytracing_amd.faithful import FaithfulPupil
        fp = FaithfulPupil(n, n, size=args.pupil, pad=args.pad, wavelengths=my_lams,
                           slots=args.faithful_lag + 3, **({"sweeps": args.cone_sweeps} if args.cone_sweeps else {}))
    elif faithful:
        # N > 1: the pupil sharded with the rays (halo rows + the boundary band to rank 0, no gather
        # of the hits: faithful_dist.py); rank 0 forms the map, the plane correction and the stack
        from akbraytracing_amd.faithful_dist import ShardedFaithfulPupil
        fp = ShardedFaithfulPupil(n, comm, size=args.pupil, pad=args.pad, wavelengths=lams,
                                  slots=args.faithful_lag + 2, workers=4,
                                  **({"sweeps": args.cone_sweeps} if args.cone_sweeps else {}))

    def faithful_back(timed, f):
        """The reference's pupil and PSF of the oldest front: its tilt and OPD were fused into later
        passes 1, so its rows are final; the cell pass and the pocket job start now, and the oldest
        run, once more than --faithful-lag are in flight, finishes on the back stream - griddata,
        plane correction, psf_calc, PSF - beside the next passes."""
        bs = back_stream
        with torch.cuda.stream(bs):
            out = rw.launch_back(f, stream=bs)
            d2 = out["detcenter2"]
            cs = bs
            if args.begin_stream != "back" and world == 1:
                cs = rw._fin if args.begin_stream == "fin" else rw._copy
                ready = torch.cuda.Event()
                ready.record(bs)
                cs.wait_event(ready)
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cs)
            tickets.append(fp.begin(d2[1], d2[2], out["wave2"], stream=cs))
            if timed:
                e1.record(cs)
                fp_events.append(("begin", e0, e1))
            # by count alone (every rank finishes the same runs, N > 1: collectives): with
            # --faithful-lag runs in flight after every step, the timed steps finish exactly as many
            # runs as they begin (faithful_finishes_timed == steps)
            while len(tickets) > args.faithful_lag:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
                pe = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) \
                    if timed and rank == 0 else None
                t = tickets.pop(0)
                fp.finish(t, stream=bs, events=ev, psf_events=pe)
                finished.append(t)
                if len(finished) > 1024:  # (the error log keeps 8192 runs: check the ones already done)
                    check_finished(False)
                if timed:
                    fp_events.append(("finish", ev[0], ev[1]))
                if pe is not None:
                    psf_events.append(pe)

    def back(timed, f=None):
        """Tilt (unless already fused into the next pass 1), OPD and pupil of the oldest front (on
        the back stream, beside the next pass 1 / during the resample), then its PSF."""
        f = f if f is not None else fronts.pop(0)
        if faithful:
            return faithful_back(timed, f)
        bs = back_stream if args.back_stream else torch.cuda.current_stream()
        with torch.cuda.stream(bs):
            rw.launch_back(f, stream=bs if args.back_stream else None)
            if state["psf_done"] is not None:  # the pupil buffer is reused: wait for its last reader
                bs.wait_event(state["psf_done"])
                state["psf_done"] = None
            opd, pitch = rw.pupil(args.pupil)
            ready = torch.cuda.Event()
            ready.record(bs)
        state["pupil"] = (opd, pitch)
        run_psf(opd, pitch, ready, timed)

    def step(timed):
        # pipelined: this step's pass 1 is queued first (with --fuse, carrying the previous step's
        # tilt), the previous step's OPD / pupil / PSF right behind it, so the GPU works through
        # them while the host does the resample; each step still traces, tilts, reduces and
        # transforms one full grid - of its own system
        i = nsteps[0]
        nsteps[0] += 1
        kw = dict(geometry=sys_of(i), next_geometry=sys_of(i + 1))
        if args.fuse >= 2 and len(fronts) == 3:  # three steps in flight: tilt k-2, OPD k-3
            old = fronts.pop(0)
            fronts.append(rw.launch_front(overlap=lambda: back(timed, old), fuse=fronts[0], fuse_opd=old, **kw))
        elif args.fuse >= 2 and len(fronts) == 2:  # filling the pipeline
            fronts.append(rw.launch_front(fuse=fronts[0], **kw))
        elif args.fuse >= 2:
            fronts.append(rw.launch_front(**kw))
        elif fronts and args.fuse:
            prev = fronts.pop(0)
            fronts.append(rw.launch_front(overlap=lambda: back(timed, prev), fuse=prev, **kw))
        else:
            fronts.append(rw.launch_front(overlap=(lambda: back(timed)) if fronts else None, **kw))

    from akbraytracing_amd import device as DEVM

    step_log = []

    def timed_steps(k):
        comm.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hm = []
        evs = []
        if args.step_log:
            e_start = torch.cuda.Event(enable_timing=True)
            e_start.record()
        for _ in range(k):
            h0, w0 = time.perf_counter(), DEVM.host_wait_s()
            step(True)
            # (host time issuing the step, of it blocked on events / the pocket job)
            hm.append(((time.perf_counter() - h0) * 1e3, (DEVM.host_wait_s() - w0) * 1e3))
            if args.step_log:
                em, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                em.record()
                eb.record(back_stream)
                evs.append((em, eb))
        torch.cuda.synchronize()
        comm.barrier()
        el = time.perf_counter() - t0
        if args.step_log:
            step_log.clear()
            step_log.extend([round(e_start.elapsed_time(em), 4), round(e_start.elapsed_time(eb), 4),
                             round(h, 4), round(w, 4)] for (em, eb), (h, w) in zip(evs, hm))
        return el, hm

    # first use of every kernel, the pocket workers and the pinned buffers of the chain, before any
    # step: one run and its faithful pupil on their own (outside every timed region; a fresh
    # process otherwise pays those first launches inside the driver's short W / K form)
    if fp is not None:
        o0 = rw.run(geometry=sys_of(0), next_geometry=sys_of(1))
        d20 = o0["detcenter2"]
        if world == 1:
            t0 = fp.begin(d20[1], d20[2], o0["wave2"], stream=back_stream)
            fp.finish(t0, stream=back_stream)
            t0.check()
        else:
            fp.run(d20[1], d20[2], o0["wave2"], stream=back_stream)
        del o0, d20
        torch.cuda.synchronize()

    # the driver's form without the clock ramp, in the same process: W warm-up steps, K timed
    no_ramp_ms = None
    if args.ramp_ms > 0 and not args.no_ramp_form:
        for _ in range(args.warmup):
            step(False)
        el0, _ = timed_steps(args.steps)
        t = comm.allreduce_max(torch.tensor([el0], dtype=torch.float64, device=dev))
        no_ramp_ms = float(t.item()) / args.steps * 1e3
        rw.kernel_events = None
        rw.pass1_events = None
        fp_events.clear()
        psf_events.clear()

    ramp_steps = 0
    if args.ramp_ms > 0:
        torch.cuda.synchronize()
        r0 = time.perf_counter()
        while True:  # in chunks of 8 steps, every rank going on while any rank's time is short
            for _ in range(8):
                step(False)
            ramp_steps += 8
            torch.cuda.synchronize()
            more = torch.tensor([float((time.perf_counter() - r0) * 1e3 < args.ramp_ms)],
                                dtype=torch.float64, device=dev)
            if float(comm.allreduce_max(more).item()) == 0.0:
                break
    for _ in range(args.warmup):
        step(False)
    rw.kernel_events = []
    rw.pass1_events = []
    fp_events.clear()
    psf_events.clear()
    # host_ms: host time spent issuing each step (its waits included): is the host the limit?
    fin0 = fp.finished if fp is not None else 0
    from akbraytracing_amd import _lib as LIBM
    if fp is not None and world == 1:  # HIP events around each patch launch of the timed steps
        LIBM.check(LIBM.lib().akb_gd_patch_timing(1))
    el, host_ms = timed_steps(args.steps)
    finishes_timed = (fp.finished - fin0) if fp is not None else None
    patch = None
    patch_launch_ms = []
    if fp is not None and world == 1:
        LIBM.check(LIBM.lib().akb_gd_patch_timing(0))  # (stops new records; the queued ones still land)
        pms = (ctypes.c_float * 1024)()
        pcells = (ctypes.c_int * 1024)()
        k = LIBM.lib().akb_gd_patch_times(pms, pcells, 1024)
        if k < 0:
            LIBM.check(k)
        if k > 0:
            K = fp.sweeps
            W = 2 * K + 4
            S = next(s2 for s2 in range((K + 1) // 2, K + 1)
                     if (W - 2) ** 2 + (W - 2 * s2 - 2) ** 2 + 4 <= 1024)
            patch = faithful_roofline(list(pms[:k]), int(pcells[k - 1]), K, S)
            patch_launch_ms = list(pms[:k])
            ph = (ctypes.c_ulonglong * 10)()
            LIBM.check(LIBM.lib().akb_gd_patch_phases(ph))
            tot = ph[0] + ph[1] + ph[2]
            if tot:  # workgroup 0's wall clock (10 ns ticks) in its steps' phases
                patch["workgroup0_phases"] = {"setup_frac": ph[0] / tot, "sweeps_frac": ph[1] / tot,
                                              "rest_frac": ph[2] / tot, "steps": int(ph[3]),
                                              "us_per_step": tot * 0.01 / max(int(ph[3]), 1)}
            if ph[7]:  # the band sweeps' workgroups (diagnostics): with a tile (and its ring share), ring only
                patch["band_workgroups"] = {"tile_avg_us": ph[6] * 0.01 / ph[7], "tile_max_us": ph[9] * 0.01,
                                            "ring_only_avg_us": ph[4] * 0.01 / ph[5] if ph[5] else None,
                                            "ring_only_max_us": ph[8] * 0.01 if ph[5] else None}
    while fronts:  # the last front's back half (outside the timed region, like the first one's)
        back(False)
    while tickets:
        t = tickets.pop(0)
        fp.finish(t, stream=back_stream)
        finished.append(t)
    torch.cuda.synchronize()
    faithful_checked = None
    if faithful:  # every run's own error words (the reference's raises), read now that nothing waits on them
        check_finished(True)
        faithful_checked = checked["runs"]
    psf_alone_ms = psf_device_ms = None
    if rank == 0:  # the PSF's own wall time, nothing beside it (the last pupil: rw.pupil is collective)
        opd, pitch = (fp.post["opd"], None) if faithful else state["pupil"]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            psf_stack(opd, None, my_lams, None, pitch=pitch, pad_factor=args.pad, out=psf_out.get("psf"))
        b.record()
        b.synchronize()
        psf_alone_ms = a.elapsed_time(b) / 10
        # the same ten calls with the device held back by a spin kernel while the host queues them:
        # the device's own time per transform (measured: 32.8 vs 33.5 us wall at 2048^2 - the host
        # keeps ahead of the three launches per call)
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda.synchronize()
            torch.cuda._sleep(20_000_000)
            a2, b2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a2.record()
            for _ in range(10):
                psf_stack(opd, None, my_lams, None, pitch=pitch, pad_factor=args.pad, out=psf_out.get("psf"))
            b2.record()
            b2.synchronize()
            psf_device_ms = a2.elapsed_time(b2) / 10
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    t = comm.allreduce_max(t)
    el = float(t.item())
    inter_rank = rw.intersections_per_run() * args.steps
    tot = torch.tensor([float(inter_rank)], dtype=torch.float64, device=dev)
    total_inter = float(comm.allreduce_sums(tot).item())
    # one run on its own, host wait included (what a caller that needs each result before the next
    # trace sees); collective at N > 1, so every rank runs it
    last_out, single_ms = None, None
    if not args.no_extras:
        single = []
        for i in range(5):
            comm.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            last_out = rw.run(geometry=sys_of(i), next_geometry=sys_of(i + 1))
            torch.cuda.synchronize()
            single.append((time.perf_counter() - t1) * 1e3)
        st = comm.allreduce_max(torch.tensor([sorted(single)[2]], dtype=torch.float64, device=dev))
        single_ms = float(st.item())

    # steps with the reference's own PSF through the host-synchronous drop-ins: each step traces a
    # system (run()) and forms its faithful PSF (faithful_psf: wave_pupil + psf_calc), nothing
    # overlapped across steps (the pipelined faithful steps are the timed region itself)
    faithful_steps = None
    if world == 1 and not args.no_extras and not faithful:
        ft = []
        for i in range(args.faithful_steps + 2):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            o = rw.run(geometry=sys_of(i), next_geometry=sys_of(i + 1))
            faithful_psf(o, rw.n, args.pupil)
            torch.cuda.synchronize()
            if i >= 2:
                ft.append((time.perf_counter() - t1) * 1e3)
        ms = sorted(ft)[len(ft) // 2]
        faithful_steps = {"ms_per_step": ms, "steps": len(ft),
                          "intersections_per_s": rw.intersections_per_run() / (ms * 1e-3),
                          "what": "run() (trace, resample, tilt, OPD) + griddata(cubic) of Wave2 -> nanmean -> plane "
                                  f"correction -> psf_calc on the {args.pupil}^2 grid, one system per step, median"}

    # N > 1: one faithful pupil + PSF on its own through the sharded route (halo rows + band to rank
    # 0, no gather of the hits; collective: wall time between barriers, median of 3)
    faithful_dist_ms = None
    if world > 1 and last_out is not None and faithful:
        ft = []
        d2 = last_out["detcenter2"]
        for _ in range(3):
            comm.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            fp.run(d2[1], d2[2], last_out["wave2"])
            torch.cuda.synchronize()
            comm.barrier()
            ft.append((time.perf_counter() - t1) * 1e3)
        faithful_dist_ms = sorted(ft)[1]

    stage = None
    if world == 1 and not args.no_extras:
        stage = stage_api(rw, geom, dev)

    # N > 1: every rank's median faithful finish (device time on its back stream, in the timed steps):
    # rank 0's excess over the others is the band owner's tail inside the step (rank0_tail below)
    tail_in_step = None
    if world > 1 and faithful:
        mine = sorted(a.elapsed_time(b) for k, a, b in fp_events if k == "finish")
        v = torch.zeros(world, dtype=torch.float64, device=dev)
        v[rank] = mine[len(mine) // 2] if mine else float("nan")
        v = comm.allreduce_sums(v).cpu().numpy()
        others = sorted(float(x) for x in v[1:])
        tail_in_step = {"rank0_finish_ms": float(v[0]), "other_ranks_finish_ms_median": others[len(others) // 2],
                        "other_ranks_finish_ms_max": others[-1],
                        "rank0_tail_ms": float(v[0]) - others[len(others) // 2],
                        "what": "median device time of a faithful finish per rank in the timed steps (HIP events "
                                "on its back stream, sharing the GPU with its passes); rank 0 adds the band "
                                "iteration, the post and the PSF"}

    if rank != 0:
        return
    k_ms = [a.elapsed_time(b) for a, b in rw.kernel_events] if rw.kernel_events else [float('nan')]
    k_avg = sum(k_ms) / len(k_ms)
    psf_ms = sum(a.elapsed_time(b) for a, b in psf_events) / max(len(psf_events), 1)
    # pass 1 (fused with run k-2's tilt and run k-3's OPD at --fuse 2): its own HIP events
    p1 = [(a.elapsed_time(b), ft, fo) for a, b, ft, fo in (rw.pass1_events or [])]
    roof_p1 = pass1_roofline(p1, rw.n_local, read_profile()[0] if args.config != "c2" else {}, args.fuse)
    # the faithful chain's device time per step on the back stream (cell pass + finish), and the
    # finishes alone (griddata, plane correction, psf_calc, PSF), sharing the GPU with the passes
    fp_begin = [a.elapsed_time(b) for k, a, b in fp_events if k == "begin"]
    fp_fin = [a.elapsed_time(b) for k, a, b in fp_events if k == "finish"]
    launch_bytes = PASS2_BYTES_PER_RAY * rw.n_local
    achieved = launch_bytes / (k_avg * 1e-3) / 1e9
    prof, prof_file, prof_ok = read_profile()
    # the profile describes the 4-mirror pass-2 kernel (C3's): no PMC fields for the KB pair
    pk = prof.get("kernels", {}).get("pass2", {}) if prof_ok and args.config != "c2" else {}
    inter_launch = len(geom.mirrors) * rw.n_local  # pass 2's intersections per launch
    # VALU-issue roofline of pass 2: the chip issues at most SIMDS / 4 wave-instructions per clock;
    # with the profiled instructions per intersection that caps the intersection rate
    vpi = (pk["valu_wave_instructions_per_launch"] / pk["intersections_per_launch"]
           if pk.get("valu_wave_instructions_per_launch") and pk.get("intersections_per_launch") else None)
    clock = pk.get("effective_clock_ghz") if pk else None
    issue_peak = (SIMDS / 4 * clock * 1e9 / vpi) if vpi and clock else None
    issue_achieved = inter_launch / (k_avg * 1e-3)
    out = {
        "metric": METRIC,
        "value": total_inter / el,
        "unit": "intersections/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "clock_ramp": {"ms": args.ramp_ms, "untimed_steps": ramp_steps},
        "ms_per_step": el / args.steps * 1e3,
        # the same K steps timed in this process after the W warm-up steps alone, before the clock
        # ramp: the driver's plain W / K form (null with --no-ramp-form or --ramp-ms 0)
        "ms_per_step_no_ramp": no_ramp_ms,
        "untimed_steps_before_timing": (args.warmup + (args.warmup + args.steps if no_ramp_ms else 0) + ramp_steps),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: deterministic ray grid through the reference's "
                + ("KB" if args.config == "c2" else "AKB") + " geometry (recorded fixture)",
        "config": {
            "workload": workload_label(args.config, world, faithful),
            "rays_per_gpu": rw.n_local, "rays_total": n * n, "grid": n, "v_rows_per_rank": round(shard.count / n, 1),
            "mirrors": len(geom.mirrors), "systems_cycled": len(systems),
            "intersections_per_step": 2 * len(geom.mirrors) * n * n,
            "psf": f"{args.pupil}^2 pupil x pad {args.pad} -> {len(lams)} x {args.pupil * args.pad}^2 complex128 "
                   "DFT (pruned)" + (f", wavelength-sharded over {min(world, len(lams))} ranks" if world > 1 and
                                     len(lams) > 1 else ""),
            "parallelism": f"ray-row shards x{world}",
            "reserved_cus": args.reserve_cus,
        },
        # the host's share of a step (medians over the timed steps): its whole time per step, the part
        # blocked on the device (event waits) or on the pocket workers, and the rest - the host's own
        # issue cost (launch calls, the resample, Python). A step time near host_pure_issue would mean
        # the host bounds the step; near the waits' sum, the device does
        "host_issue_ms_per_step": sorted(h for h, _ in host_ms)[len(host_ms) // 2],
        "host_wait_ms_per_step": sorted(w for _, w in host_ms)[len(host_ms) // 2],
        "host_pure_issue_ms_per_step": sorted(h - w for h, w in host_ms)[len(host_ms) // 2],
        "pupil": ("faithful: each step's PSF from the reference's own pupil - griddata(cubic) of Wave2 on the "
                  f"{n}^2 hits (cone solve, {fp.K if world > 1 else fp.sweeps} Chebyshev sweeps), nanmean removal, "
                  "plane correction, psf_calc (rotation, rotate_with_nan, pad 16) - pipelined on the back stream "
                  + ("(akbraytracing_amd/faithful.py)" if world == 1 else
                     f"(akbraytracing_amd/faithful_dist.py: each rank grids its own rows, halo of {fp.K + 3} rows "
                     f"from its neighbours, the boundary band ({sum(fp.plan.band_count(r) for r in range(world))} "
                     f"hits) to rank 0)") if faithful else
                  "stand-in: RayWave.pupil's ray-index sampler (up to 0.098 nm from the reference's Clough-Tocher)"),
        # faithful runs finished inside the timed region (count-based lag: equal to steps) and runs
        # whose own error words were checked after it
        "faithful_finishes_timed": finishes_timed,
        "faithful_runs_checked": faithful_checked,
        "cone_guard_trips": checked["guard_trips"] if faithful else None,
        "faithful_chain_ms": ((sum(fp_begin) + sum(fp_fin)) / max(len(fp_fin), 1)) if fp_fin else None,
        # the faithful chain's dominant kernel: the cone solve's patches (in the timed steps)
        "roofline_faithful": patch,
        "faithful_finish_ms": (sum(fp_fin) / len(fp_fin)) if fp_fin else None,
        "psf_ms": psf_ms if psf_events else None,
        "psf_alone_ms": psf_alone_ms,
        "psf_device_ms": psf_device_ms,
        # the PSF's compulsory HBM traffic is its output (the pupil is 128 KB): intensity planes
        "psf_alone_output_gbs": (len(my_lams) * (args.pupil * args.pad) ** 2 * 8 / (psf_alone_ms * 1e-3) / 1e9
                                 if psf_alone_ms else None),
        "pass2_kernel_ms": k_avg,
        # the contract's HBM roofline for the dominant kernel (pass 2, k_chain_sink with its fixed
        # output set): algorithmic bytes over this run's event time. It moves 14 B per
        # intersection, so HBM does not bound it; roofline_issue below is its real ceiling
        "roofline": {
            "kernel": "k_chain_sink<grid,opl,point,fixed> (pass 2)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": pk.get("hbm_bytes_per_launch"),
            "algorithmic_bytes_per_launch": launch_bytes,
        },
        # the fused pass 1 (the step's longest trace kernel at --fuse 2)
        "roofline_pass1": roof_p1,
        # what bounds pass 2: VALU issue. Peak = intersections/s the chip would reach issuing one
        # wave-instruction per SIMD every 4 cycles at the profiled clock, with the profiled VALU
        # wave-instructions per intersection; frac = this run's rate over it
        "roofline_issue": {
            "kernel": pk.get("kernel"),
            "bound": "valu-issue",
            "achieved": issue_achieved,
            "peak": issue_peak,
            "unit": "intersections/s",
            "frac": issue_achieved / issue_peak if issue_peak else None,
            "valu_wave_instructions_per_intersection": vpi,
            "non_fp64_share": pk.get("non_fp64_share"),
            "effective_clock_ghz": clock,
            "issue_frac_profiled": pk.get("issue_frac"),
            "valu_busy_pct_profiled": pk.get("valu_busy_pct"),
        },
        "roofline_fp64": {
            "bound": "fp64-valu",
            "achieved": (pk["fp64_flops_per_launch"] / (k_avg * 1e-3) / 1e12) if pk else None,
            "peak": FP64_VALU_PEAK_TFS,
            "unit": "TFLOP/s",
            "frac": (pk["fp64_flops_per_launch"] / (k_avg * 1e-3) / 1e12 / FP64_VALU_PEAK_TFS) if pk else None,
        },
        # where the PMC-derived fields above come from (null when no profile matches the sources)
        "profile": {"file": prof_file, "matches_sources": prof_ok, "git_head": prof.get("git_head"),
                    "kernel": pk.get("kernel")},
        # provenance: sha256 of the kernel sources compiled into the loaded libakb_hip.so (the
        # loader refuses a library whose hash differs from this tree's, akbraytracing_amd/_lib.py)
        "lib_sources_hash": _lib_hash(),
    }
    if single_ms is not None:
        out["single_run_ms"] = single_ms
    if faithful_dist_ms is not None:
        out["faithful_psf_chain_ms"] = faithful_dist_ms
        out["faithful_psf_route"] = (f"sharded over the {world} ray shards (faithful_dist.py): halo rows and the "
                                     "boundary band move, not the hits; one run alone, between barriers")
    if tail_in_step is not None:
        out["rank0_tail"] = tail_in_step
    if world > 1:
        out["note_multi_gpu"] = ("shards are aligned to numpy's 8192-element sum buffers and the ranks' buffer sums "
                                 "are chained in numpy's order: N ranks give one process's bits "
                                 "(tests/test_c4_gpu.py, tests/test_dist_gpu.py)")
    if world == 1 and last_out is not None:
        out["huygens_pairs_per_s"] = huygens_rate(last_out)
        chain_ms, maps_ms = faithful_psf_chain(rw, last_out, args.pupil)
        # the PSF of the reference's own pupil: griddata(cubic) -> nanmean -> plane correction ->
        # psf_calc on this trace's 1e7 detector-2 hits
        out["faithful_psf_chain_ms"] = chain_ms
        out["faithful_wave_maps_psf_ms"] = maps_ms
        if fp is not None:
            # one run's pipelined chain on its own (begin + pocket job + finish, device synchronised):
            # its latency, not its share of a step
            d2 = last_out["detcenter2"]
            ft = []
            for _ in range(5):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                fp.run(d2[1], d2[2], last_out["wave2"])
                torch.cuda.synchronize()
                ft.append((time.perf_counter() - t1) * 1e3)
            out["faithful_pipelined_single_ms"] = sorted(ft)[2]
        if faithful_steps is not None:
            out["faithful_step"] = faithful_steps
        if stage is not None:
            out["stage_api"] = stage
        if not args.no_extras and args.config == "c3":
            out["rank0_tail"] = rank0_tail()
    if step_log:
        out["step_log"] = {"columns": ["main_done_ms", "back_done_ms", "host_ms", "host_wait_ms"],
                           "steps": step_log,
                           # the same timed steps' kernels in launch order (HIP events)
                           "pass1_ms": [round(a.elapsed_time(b), 4) for a, b, _, _ in (rw.pass1_events or [])],
                           "pass2_ms": [round(a.elapsed_time(b), 4) for a, b in (rw.kernel_events or [])],
                           "patch_ms": [round(float(x), 4) for x in patch_launch_ms]}
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, gdict)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
