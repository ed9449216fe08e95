"""Summarise the Huygens stage's rocprofv3 outputs (scripts/gpu_huygens_prof.sh) into profiles/:

    python scripts/summarize_huygens.py r02b

<tag>_huygens_kernel_stats.csv (the kernel-trace summary of scripts/bench_huygens.py) and
<tag>_huygens.json: for the M2 -> image launch (1e7 sources x 65^2 targets, BASELINE configs[1]'s
stage shape, the launch with the most VALU work) the pairs, duration, VALU wave-instructions per
pair, the FP64 mix and rate, VALU busy and the issue fraction, each counter from its own pass
(medians over the launches of that shape).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out")
DST = os.path.join(ROOT, "profiles")
SIMDS, XCDS, CUS = 1024, 8, 256
FP64_PEAK_TFS = 78.6


def main(tag, sources=10004569, targets=4225):
    os.makedirs(DST, exist_ok=True)
    stats = os.path.join(SRC, "hprof", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(DST, f"{tag}_huygens_kernel_stats.csv"))
    # the stats file averages every k_huygens launch (both stage shapes): take this shape's launches
    # from the trace (the few-target stage has the smallest grid)
    tr = [r for r in csv.DictReader(open(os.path.join(SRC, "hprof", "run_kernel_trace.csv")))
          if r["Kernel_Name"].startswith("akb::k_huygens(")]
    gsz = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])  # noqa: E731
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
    # the M2 -> image launches: the longest ones (split over sources; the source -> M1 stage is short)
    shape = gsz(max(tr, key=dur))
    td = sorted(dur(r) for r in tr if gsz(r) == shape)
    trace_ns = float(td[len(td) // 2])
    # per counter: values of the big launches (grid of the M2 -> image shape: the largest VALU count)
    vals = collections.defaultdict(list)
    durs = []
    for i in range(1, 20):
        f = os.path.join(SRC, f"hpmc_{i}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("akb::k_huygens(")]
        # the M2 -> image launch: the longest dispatch of the pass
        big = max(rows, key=lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))["Grid_Size"]
        for r in rows:
            if r["Grid_Size"] == big:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                if r["Counter_Name"] in ("GRBM_GUI_ACTIVE",):
                    durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
    pairs = sources * targets
    valu = med["SQ_INSTS_VALU"]
    f64 = {k: med.get(f"SQ_INSTS_VALU_{k.upper()}_F64", 0.0) for k in ("add", "mul", "fma", "trans")}
    f64_total = sum(f64.values())
    flops = 64 * (f64["add"] + f64["mul"] + f64["trans"] + 2 * f64["fma"])
    cycles = med["GRBM_GUI_ACTIVE"] / XCDS
    pmc_ns = sorted(durs)[len(durs) // 2]
    import hashlib
    src = os.path.join(ROOT, "akbraytracing_amd", "csrc", "akb_huygens.hip")
    out = {
        "tag": tag,
        "sources_sha256": hashlib.sha256(open(src, "rb").read()).hexdigest(),
        "command": "python3 scripts/bench_huygens.py --reps 2 (kernel trace); --reps 1 per PMC pass",
        "kernel": "akb::k_huygens (M2 -> 65x65 image grid: 1e7 sources, 4225 targets, split over sources)",
        "sources": sources, "targets": targets, "pairs_per_launch": pairs,
        "median_duration_ns_kernel_trace": trace_ns,
        "duration_ns_pmc_runs": pmc_ns,
        "pairs_per_s": pairs / (trace_ns * 1e-9) if trace_ns else None,
        "effective_clock_ghz": cycles / pmc_ns,
        "valu_wave_instructions_per_launch": valu,
        "valu_lane_ops_per_pair": 64 * valu / pairs,
        "fp64_wave_instructions_per_launch": f64_total,
        "fp64_by_kind": f64,
        "fp64_lane_ops_per_pair": 64 * f64_total / pairs,
        "non_fp64_share": (valu - f64_total) / valu,
        "int32_valu": med.get("SQ_INSTS_VALU_INT32"),
        "salu": med.get("SQ_INSTS_SALU"),
        "lds_instructions": med.get("SQ_INSTS_LDS"),
        "fp64_flops_per_launch": flops,
        "fp64_tflops": flops / (trace_ns * 1e-9) / 1e12 if trace_ns else None,
        "fp64_frac_of_peak": flops / (trace_ns * 1e-9) / 1e12 / FP64_PEAK_TFS if trace_ns else None,
        "fp64_peak_tflops": FP64_PEAK_TFS,
        "valu_busy_pct": 100.0 * med["SQ_ACTIVE_INST_VALU"] / CUS / cycles,
        "issue_frac": valu * 4 / SIMDS / cycles,
        "bound": "VALU issue (FP64 sqrt / reciprocal / sincos per pair; sources stream from LDS)",
    }
    with open(os.path.join(DST, f"{tag}_huygens.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02b")
