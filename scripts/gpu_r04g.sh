#!/bin/bash
# Round-4 GPU pass 7: where the register patch kernel's cycles go (AKB_GD_PATCH_CLOCK per-phase
# cycle sums), and the next-cell register prefetch (AKB_GD_PATCH_PREFETCH) against the plain load.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
AKB_GD_PATCH_CLOCK=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 3 > gpurun_out/r04g_clk.log 2>&1
rc=$?; grep AKB_GD_PATCH_CLOCK gpurun_out/r04g_clk.log | tail -2; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
AKB_GD_PATCH_CLOCK=1 AKB_GD_PATCH_PREFETCH=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 3 > gpurun_out/r04g_clkpf.log 2>&1
rc=$?; grep AKB_GD_PATCH_CLOCK gpurun_out/r04g_clkpf.log | tail -2; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8 -o run -- \
    python3 scripts/micro_faithful.py --reps 10 --out /tmp/mf_a.npz > gpurun_out/r04g_micro.log 2>&1
rc=$?; tail -1 gpurun_out/r04g_micro.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/prof8/run_kernel_stats.csv | head -6; rm -f gpurun_out/prof8/run_kernel_trace.csv
AKB_GD_PATCH_PREFETCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof9 -o run -- \
    python3 scripts/micro_faithful.py --reps 10 --out /tmp/mf_b.npz > gpurun_out/r04g_micro_pf.log 2>&1
rc=$?; tail -1 gpurun_out/r04g_micro_pf.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/prof9/run_kernel_stats.csv | head -6; rm -f gpurun_out/prof9/run_kernel_trace.csv
python3 -c "
import numpy as np
a, b = np.load('/tmp/mf_a.npz'), np.load('/tmp/mf_b.npz')
print('pf == plain:', {k: bool(np.array_equal(a[k], b[k], equal_nan=True)) for k in a.files})"
