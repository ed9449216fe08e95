#!/bin/bash
# Round-4 GPU pass 8: the pipeline's next box through registers (A/B: by LDS DMA), parity tests,
# per-phase cycles, kernel times, outputs against the 256-thread patch kernel, then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_faithful_gpu.py tests/test_faithful_dist_gpu.py \
  -m gpu -x -v -s --timeout 300 --timeout-method thread -k "${PYTEST_K:-cone or gradient or faithful or sharded or griddata or claim}" \
  > gpurun_out/r04h_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04h_pytest.log; [ $rc -eq 0 ] || exit $rc
AKB_GD_PATCH_CLOCK=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 2 > gpurun_out/r04h_clk.log 2>&1
rc=$?; grep AKB_GD_PATCH_CLOCK gpurun_out/r04h_clk.log | tail -1; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
AKB_GD_PATCH_CLOCK=1 AKB_GD_PATCH_DMA=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 2 > gpurun_out/r04h_clkpf.log 2>&1
rc=$?; grep AKB_GD_PATCH_CLOCK gpurun_out/r04h_clkpf.log | tail -1; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o run -- \
    python3 scripts/micro_faithful.py --reps 10 --out /tmp/mf_a.npz > gpurun_out/r04h_micro.log 2>&1
rc=$?; tail -1 gpurun_out/r04h_micro.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/prof10/run_kernel_stats.csv > gpurun_out/r04h_k.txt; head -8 gpurun_out/r04h_k.txt; rm -f gpurun_out/prof10/run_kernel_trace.csv
AKB_GD_PATCH_DMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof11 -o run -- \
    python3 scripts/micro_faithful.py --reps 10 --out /tmp/mf_b.npz > gpurun_out/r04h_micro_pf.log 2>&1
rc=$?; tail -1 gpurun_out/r04h_micro_pf.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/prof11/run_kernel_stats.csv > gpurun_out/r04h_kpf.txt; head -3 gpurun_out/r04h_kpf.txt; rm -f gpurun_out/prof11/run_kernel_trace.csv
AKB_GD_PATCH_V1=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 3 --out /tmp/mf_c.npz > gpurun_out/r04h_micro_v1.log 2>&1
rc=$?; tail -1 gpurun_out/r04h_micro_v1.log; fatal $rc && exit $rc
python3 -c "
import numpy as np
a, b, c = np.load('/tmp/mf_a.npz'), np.load('/tmp/mf_b.npz'), np.load('/tmp/mf_c.npz')
print('pf == plain:', {k: bool(np.array_equal(a[k], b[k], equal_nan=True)) for k in a.files})
print('v1 == plain:', {k: bool(np.array_equal(a[k], c[k], equal_nan=True)) for k in a.files})"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err
rc=$?; fatal $rc && exit $rc
python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/r04h_bench.json') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('value', 'ms_per_step', 'faithful_chain_ms', 'faithful_finish_ms', 'psf_ms', 'host_issue_ms_per_step')})"
exit $rc
