"""Turn the rocprofv3 outputs a gpurun call left under gpurun_out/ into the committed summaries
under profiles/: kernel stats, PMC per kernel, and <tag>_roofline.json, the per-launch figures
bench.py reports for the two chain kernels (pass 2 and the fused pass 1 + tilt + OPD).

    python scripts/summarize_profiles.py r02a

Every PMC pass is its own rocprofv3 run (scripts/gpu_pmc.sh), with each FP64 counter alone in
its pass. HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KB; on gfx950
FETCH_SIZE counts half the bytes of a wide streaming read, so it is doubled; WRITE_SIZE is taken
as is. FP64 work: SQ_INSTS_VALU_{ADD,MUL,TRANS}_F64 + 2 x FMA_F64 wave instructions x 64 lanes.

Issue roofline: a wave64 VALU instruction occupies its SIMD for 4 cycles (16 lanes per SIMD, FP64
at full rate on CDNA4), so a launch needs at least SQ_INSTS_VALU x 4 / 1024 SIMD-cycles; the
issue fraction is that over the launch's own cycles (GRBM_GUI_ACTIVE / 8 XCDs, in the same
serialised PMC run, whose timestamps also give the clock).

The summary records the sha256 of the kernel sources it describes; bench.py uses its figures only
while the sources still hash the same (otherwise it reports them as null and names the file).
"""
import collections
import csv
import hashlib
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out")
DST = os.path.join(ROOT, "profiles")
TRACE_SOURCES = ["akbraytracing_amd/csrc/akb_trace.hip", "akbraytracing_amd/csrc/akb_common.h",
                 "akbraytracing_amd/csrc/akb_pairwise.h", "include/akb_raytrace.h"]
# the kernels bench.py reports: (key, kernel-name prefix, algorithmic HBM bytes per ray, rays label)
KERNELS = [
    ("pass2", "void akb::k_chain_sink<true, true", 56,
     "pass 2: 4 mirrors + OPL + detector + 2 arctan; writes last hit, exit direction, OPL (56 B/ray)"),
    ("pass1_fused", "void akb::k_chain_tilt<4, true>", 56 + 32 + 48,
     "pass 1 of run k (4 mirrors) + tilt of run k-2 (reads 56 B, writes det2 + total2, 32 B) "
     "+ OPD of run k-3 (reads 32 B, writes 16 B)"),
]
# the faithful chain's kernels (akb_griddata.hip): the cone solve's patch kernel and band sweep
GD_SOURCES = ["akbraytracing_amd/csrc/akb_griddata.hip", "akbraytracing_amd/csrc/akb_common.h",
              "akbraytracing_amd/csrc/akb_pairwise.h", "include/akb_raytrace.h"]
GD_KERNELS = [("cone_patch", "akb::(anonymous namespace)::k_gd_cone_patch("),
              ("cone_band", "akb::(anonymous namespace)::k_gd_cone_band(")]
SIMDS = 1024  # 256 CUs x 4 SIMDs
XCDS = 8


def sources_sha256(root=ROOT, sources=None):
    h = hashlib.sha256()
    for rel in (TRACE_SOURCES if sources is None else sources):
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def pmc_table():
    """kernel -> counter -> median value; kernel -> median duration (ns) in the PMC runs"""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for i in range(1, 40):
        f = os.path.join(SRC, f"pmc_{i}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # medians: a dispatch that shares the GPU with another process's work (or the profiler's own
    # first-launch setup) inflates GRBM_GUI_ACTIVE and the duration of that one sample
    med = lambda v: sorted(v)[len(v) // 2]
    return ({k: {c: med(v) for c, v in d.items()} for k, d in agg.items()}, {k: med(v) for k, v in dur.items()})


def kernel_summary(name, d, pmc_ns, trace_ns, bytes_per_ray, n_rays, label):
    fetch = d.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = d.get("WRITE_SIZE", 0.0) * 1024
    add, mul = d.get("SQ_INSTS_VALU_ADD_F64", 0.0), d.get("SQ_INSTS_VALU_MUL_F64", 0.0)
    fma, trans = d.get("SQ_INSTS_VALU_FMA_F64", 0.0), d.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    f64 = add + mul + fma + trans
    valu = d.get("SQ_INSTS_VALU")
    cycles = d.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
    clock = cycles / pmc_ns if pmc_ns else None
    inter = 4 * n_rays  # four mirrors per ray in either kernel
    out = {
        "kernel": name,
        "what": label,
        "rays_per_launch": n_rays,
        "intersections_per_launch": inter,
        "algorithmic_bytes_per_launch": bytes_per_ray * n_rays,
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "avg_duration_ns_kernel_trace": trace_ns,
        "avg_duration_ns_pmc_runs": pmc_ns,
        "effective_clock_ghz": clock,
        "valu_wave_instructions_per_launch": valu,
        "fp64_wave_instructions_per_launch": f64,
        "fp64_by_kind": {"add": add, "mul": mul, "fma": fma, "trans": trans},
        "fp64_flops_per_launch": 64 * (add + mul + trans + 2 * fma),
        "non_fp64_valu_wave_instructions_per_launch": (valu - f64) if valu else None,
        "non_fp64_share": ((valu - f64) / valu) if valu else None,
        "valu_lane_ops_per_intersection": (64 * valu / inter) if valu else None,
        "int32_valu": d.get("SQ_INSTS_VALU_INT32"),
        "int64_valu": d.get("SQ_INSTS_VALU_INT64"),
        "salu": d.get("SQ_INSTS_SALU"),
        # rocprof's VALUBusy: 100 * SQ_ACTIVE_INST_VALU / CU_NUM / (GRBM_GUI_ACTIVE per XCD)
        "valu_busy_pct": (100.0 * d["SQ_ACTIVE_INST_VALU"] / 256 / cycles
                          if d.get("SQ_ACTIVE_INST_VALU") and cycles else None),
        "issue_cycles_min": (valu * 4 / SIMDS) if valu else None,
        "issue_frac": (valu * 4 / SIMDS / cycles) if valu and cycles else None,
        # the stall diagnosis: share of wave cycles spent waiting (s_waitcnt and dependencies), and
        # the VMEM instructions in flight per wave cycle (SQ_INST_LEVEL_VMEM accumulates the level)
        "wait_any_frac": (d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
                          if d.get("SQ_WAIT_ANY") is not None and d.get("SQ_WAVE_CYCLES") else None),
        "wait_inst_any_frac": (d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]
                               if d.get("SQ_WAIT_INST_ANY") is not None and d.get("SQ_WAVE_CYCLES") else None),
        "vmem_level_per_wave_cycle": (d["SQ_INST_LEVEL_VMEM"] / d["SQ_WAVE_CYCLES"]
                                      if d.get("SQ_INST_LEVEL_VMEM") is not None and d.get("SQ_WAVE_CYCLES") else None),
    }
    if pmc_ns:
        out["fp64_tflops_pmc_run"] = out["fp64_flops_per_launch"] / pmc_ns / 1e3
    return out


def main(tag):
    os.makedirs(DST, exist_ok=True)
    stats = os.path.join(SRC, "prof", "run_kernel_stats.csv")
    dur = {}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(DST, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            dur[r["Name"]] = float(r["AverageNs"])
    pmc, pmc_dur = pmc_table()
    if pmc:
        names = sorted({c for d in pmc.values() for c in d})
        with open(os.path.join(DST, f"{tag}_pmc_summary.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "avg_ns_kernel_trace", "avg_ns_pmc_runs"] + names)
            for k, d in sorted(pmc.items(), key=lambda kv: -dur.get(kv[0], 0)):
                w.writerow([k, dur.get(k, ""), pmc_dur.get(k, "")] + [d.get(c, "") for c in names])
    n_rays = int(os.environ.get("AKB_PROFILE_RAYS", 3163 * 3163))
    try:
        head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True,
                              text=True).stdout.strip()
    except Exception:
        head = None
    summary = {"tag": tag, "sources": TRACE_SOURCES, "sources_sha256": sources_sha256(), "git_head": head,
               "command": os.environ.get("AKB_PROFILE_CMD", "python3 bench.py --steps 20 --warmup 30 --no-cpu-baseline --no-extras"),
               "kernels": {}}
    for key, prefix, bpr, label in KERNELS:
        name = next((k for k in pmc if k.startswith(prefix)), None)
        # only from a profile of the trace kernels (scripts/gpu_pmc.sh); the faithful chain's passes
        # (scripts/gpu_pmc_faithful.sh) leave them without the issue and traffic counters
        if name is None or not all(c in pmc[name] for c in ("FETCH_SIZE", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")):
            continue
        tns = next((v for k, v in dur.items() if k.startswith(prefix)), None)
        summary["kernels"][key] = kernel_summary(name, pmc[name], pmc_dur.get(name), tns, bpr, n_rays, label)
    if summary["kernels"]:
        with open(os.path.join(DST, f"{tag}_roofline.json"), "w") as f:
            json.dump(summary, f, indent=1)
        print(json.dumps(summary, indent=1))
    gd = {"tag": tag, "sources": GD_SOURCES, "sources_sha256": sources_sha256(sources=GD_SOURCES), "git_head": head,
          "command": os.environ.get("AKB_PROFILE_CMD", ""), "kernels": {}}
    for key, prefix in GD_KERNELS:
        name = next((k for k in pmc if k.startswith(prefix)), None)
        if name is None:
            continue
        d = pmc[name]
        cycles = d.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        valu, lds = d.get("SQ_INSTS_VALU"), d.get("SQ_INSTS_LDS")
        add, mul = d.get("SQ_INSTS_VALU_ADD_F64", 0.0), d.get("SQ_INSTS_VALU_MUL_F64", 0.0)
        fma, trans = d.get("SQ_INSTS_VALU_FMA_F64", 0.0), d.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        gd["kernels"][key] = {
            "kernel": name,
            "avg_duration_ns_kernel_trace": next((v for k, v in dur.items() if k.startswith(prefix)), None),
            "avg_duration_ns_pmc_runs": pmc_dur.get(name),
            "effective_clock_ghz": cycles / pmc_dur[name] if pmc_dur.get(name) else None,
            "hbm_bytes_per_launch": d.get("FETCH_SIZE", 0.0) * 1024 * 2 + d.get("WRITE_SIZE", 0.0) * 1024,
            "valu_wave_instructions_per_launch": valu,
            "fp64_flops_per_launch": 64 * (add + mul + trans + 2 * fma),
            "lds_wave_instructions_per_launch": lds,
            "lds_bank_conflict_cycles_per_launch": d.get("SQ_LDS_BANK_CONFLICT"),
            "salu_per_launch": d.get("SQ_INSTS_SALU"),
            "valu_busy_pct": (100.0 * d["SQ_ACTIVE_INST_VALU"] / 256 / cycles
                              if d.get("SQ_ACTIVE_INST_VALU") and cycles else None),
            "issue_frac": (valu * 4 / SIMDS / cycles) if valu and cycles else None,
            "wait_any_frac": (d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
                              if d.get("SQ_WAIT_ANY") is not None and d.get("SQ_WAVE_CYCLES") else None),
            "counters": d,
        }
    if gd["kernels"]:
        with open(os.path.join(DST, f"{tag}_faithful_roofline.json"), "w") as f:
            json.dump(gd, f, indent=1)
        print(json.dumps({k: {q: v for q, v in d.items() if q != "counters"} for k, d in gd["kernels"].items()},
                         indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
