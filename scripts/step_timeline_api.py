"""Kernels, copies and the host's HIP calls of two middle steps of a traced bench run
(scripts/gpu_timeline_api.sh): device rows 'D', host rows 'H' (launches name their kernel,
waits show how long the host blocked), in µs from the step's fused pass-1 kernel start."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tla"
K = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
M = list(csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")))
A = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
name = {r["Correlation_Id"]: r["Kernel_Name"].replace("void ", "").replace("akb::", "")[:48] for r in K}
name.update({r["Correlation_Id"]: "copy " + r["Direction"][12:] for r in M})
ev = []
for r in K:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"D s{r['Stream_Id']:>2} {name[r['Correlation_Id']]}"))
for r in M:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"D s{r['Stream_Id']:>2} {name[r['Correlation_Id']]}"))
keep = {"hipEventSynchronize", "hipLaunchKernel", "hipMemcpyAsync", "hipStreamWaitEvent", "hipStreamSynchronize"}
for r in A:
    if r["Function"] in keep:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        what = r["Function"][3:]
        if r["Correlation_Id"] in name:
            what += " -> " + name[r["Correlation_Id"]]
        ev.append((s, e, "H      " + what))
ev.sort()
starts = [s for s, e, w in ev if w.startswith("D") and "k_chain_tilt" in w]
k = len(starts) // 2
for kk in (k, k + 1):
    t0, t1 = starts[kk], starts[kk + 1]
    print(f"---- step {kk}: {(t1 - t0) / 1e3:.1f} us")
    for s, e, w in ev:
        if t0 <= s < t1:
            print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} ({(e - s) / 1e3:6.1f}) {w}")
