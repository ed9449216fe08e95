"""Turn the rocprofv3 outputs a gpurun call left under gpurun_out/ into the committed summaries
under profiles/ (kernel stats, PMC per kernel, and the pass-2 chain's traffic / FP64 work per
launch that bench.py reports as roofline.traffic).

    python scripts/summarize_profiles.py r01

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KB; on gfx950
FETCH_SIZE counts half the bytes of a wide streaming read, so it is doubled; WRITE_SIZE is taken
as is. FP64 work: SQ_INSTS_VALU_{ADD,MUL,TRANS}_F64 + 2 x FMA_F64 wave instructions x 64 lanes.
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
PASS2 = "akb::k_chain_sink<true, true"


def pmc_table():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for i in range(1, 9):
        f = os.path.join(SRC, f"pmc_{i}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main(tag):
    os.makedirs(DST, exist_ok=True)
    stats = os.path.join(SRC, "prof", "run_kernel_stats.csv")
    dur = {}
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(DST, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            dur[r["Name"]] = float(r["AverageNs"])
    pmc = pmc_table()
    if pmc:
        names = sorted({c for d in pmc.values() for c in d})
        with open(os.path.join(DST, f"{tag}_pmc_summary.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "avg_ns"] + names)
            for k, d in sorted(pmc.items(), key=lambda kv: -dur.get(kv[0], 0)):
                w.writerow([k, dur.get(k, "")] + [d.get(c, "") for c in names])
    key = next((k for k in pmc if PASS2 in k), None)
    if key:
        d = pmc[key]
        fetch = d.get("FETCH_SIZE", 0.0) * 1024 * 2
        write = d.get("WRITE_SIZE", 0.0) * 1024
        f64_wave = (d.get("SQ_INSTS_VALU_ADD_F64", 0) + d.get("SQ_INSTS_VALU_MUL_F64", 0)
                    + d.get("SQ_INSTS_VALU_TRANS_F64", 0) + d.get("SQ_INSTS_VALU_FMA_F64", 0))
        flops = 64 * (d.get("SQ_INSTS_VALU_ADD_F64", 0) + d.get("SQ_INSTS_VALU_MUL_F64", 0)
                      + d.get("SQ_INSTS_VALU_TRANS_F64", 0) + 2 * d.get("SQ_INSTS_VALU_FMA_F64", 0))
        ns = next((v for k, v in dur.items() if PASS2 in k), None)
        out = {
            "kernel": key,
            "hbm_bytes_per_launch": fetch + write,
            "fetch_bytes_corrected": fetch, "write_bytes": write,
            "fp64_wave_instructions_per_launch": f64_wave,
            "fp64_flops_per_launch": flops,
            "valu_wave_instructions_per_launch": d.get("SQ_INSTS_VALU"),
            "avg_duration_ns_kernel_trace": ns,
            "effective_clock_ghz": (d.get("GRBM_GUI_ACTIVE", 0) / 8 / ns) if ns else None,
            # rocprof's VALUBusy: 100 * SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE (per XCD)
            "valu_busy_pct": (100.0 * d["SQ_ACTIVE_INST_VALU"] / 256 / (d["GRBM_GUI_ACTIVE"] / 8)
                              if d.get("SQ_ACTIVE_INST_VALU") and d.get("GRBM_GUI_ACTIVE") else None),
            "non_fp64_valu_wave_instructions_per_launch": (d.get("SQ_INSTS_VALU", 0) - f64_wave
                                                           if d.get("SQ_INSTS_VALU") else None),
            "int32_valu_wave_instructions_per_launch": d.get("SQ_INSTS_VALU_INT32"),
            "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM; WRITE_SIZE is uncalibrated for 8-B stores",
        }
        if ns:
            out["fp64_tflops"] = flops / ns / 1e3
        with open(os.path.join(DST, f"{tag}_pmc_pass2.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
