"""Print one bench step's kernel timeline from a rocprofv3 kernel trace (gpurun_out/prof).
A step starts at a pass-1 launch (k_chain<true, false, ...> or the fused k_chain_tilt)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# a step starts at its pass-1 kernel: the fused pass 1 + tilt, or (unfused) the long k_chain pass 1
big = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 50_000
idx = [i for i, r in enumerate(rows)
       if "k_chain_tilt" in r["Kernel_Name"]
       or ("k_chain<true, false" in r["Kernel_Name"] and "sink" not in r["Kernel_Name"] and big(r))]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev = None
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {gap:6.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
    prev = max(prev or 0, e)
