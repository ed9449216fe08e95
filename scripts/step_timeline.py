"""Per-step kernel timeline of a pipelined bench run (gpurun_out/tl, scripts/gpu_timeline.sh):
steps start at the fused pass-1 kernel (k_chain_tilt); prints two middle steps and the step
lengths."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tl/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_chain_tilt" in r["Kernel_Name"]]
k = len(idx) // 2
for kk in (k, k + 1):
    i0, i1 = idx[kk], idx[kk + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    print("---- step", kk, "length", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, "us")
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f} ({(e - s) / 1e3:6.1f}) q{r['Queue_Id']} {r['Kernel_Name'][:70]}")
steps = [(int(rows[idx[j + 1]]["Start_Timestamp"]) - int(rows[idx[j]]["Start_Timestamp"])) / 1e3 for j in range(len(idx) - 1)]
print("step lengths (us):", [round(s) for s in steps])
