#!/bin/bash
# Round-4 GPU pass 6: tiled cell pass + block-skipping claims; parity tests, the faithful chain
# alone under a kernel trace (new kernels vs the previous ones, same outputs), then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_faithful_gpu.py tests/test_faithful_dist_gpu.py \
  -m gpu -x -v -s --timeout 300 --timeout-method thread -k "${PYTEST_K:-griddata or cone or gradient or claim or faithful or nonuniform or sharded or default_tol or wave_maps}" \
  > gpurun_out/r04f_pytest.log 2>&1
rc=$?; tail -6 gpurun_out/r04f_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o run -- \
    python3 scripts/micro_faithful.py --out /tmp/mf_new.npz > gpurun_out/r04f_micro.log 2>&1
rc=$?; tail -2 gpurun_out/r04f_micro.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py gpurun_out/prof6/run_kernel_stats.csv; rm -f gpurun_out/prof6/run_kernel_trace.csv
AKB_GD_PATCH_ROWMAJOR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof7 -o run -- \
    python3 scripts/micro_faithful.py --reps 10 > gpurun_out/r04f_micro_rm.log 2>&1
rc=$?; tail -1 gpurun_out/r04f_micro_rm.log; fatal $rc && exit $rc
python3 scripts/kstats.py gpurun_out/prof7/run_kernel_stats.csv | head -4; rm -f gpurun_out/prof7/run_kernel_trace.csv
AKB_GD_CELLS_V1=1 AKB_GD_CLAIM_V1=1 AKB_GD_PATCH_V1=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 5 \
    --out /tmp/mf_old.npz > gpurun_out/r04f_micro_old.log 2>&1
rc=$?; tail -1 gpurun_out/r04f_micro_old.log; fatal $rc && exit $rc
python3 -c "
import numpy as np
a, b = np.load('/tmp/mf_new.npz'), np.load('/tmp/mf_old.npz')
print('new == old:', {k: bool(np.array_equal(a[k], b[k], equal_nan=True)) for k in a.files})"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err
rc=$?; fatal $rc && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --cone-sweeps 14 \
    > gpurun_out/r04f_bench14.json 2> gpurun_out/r04f_bench14.err
rc2=$?
python3 -c "
import json
for f in ('gpurun_out/r04f_bench.json', 'gpurun_out/r04f_bench14.json'):
    try:
        d = json.loads([l for l in open(f) if l.startswith('{')][-1])
        print(f, {k: d.get(k) for k in ('value', 'ms_per_step', 'ms_per_step_no_ramp', 'faithful_chain_ms', 'faithful_finish_ms', 'psf_ms', 'host_issue_ms_per_step')})
    except Exception as e:
        print(f, 'unreadable', e)
"
exit $rc2
