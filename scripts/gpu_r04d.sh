#!/bin/bash
# Round-4 GPU pass 4: the faithful chain's kernels under a kernel trace (the bench's default
# faithful step, short), plus the configs tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
final=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --ramp-ms 0 --no-ramp-form \
    > gpurun_out/r04d_prof_bench.json 2> gpurun_out/r04d_prof_bench.err
rc=$?; echo "prof exit $rc"; fatal $rc && exit $rc; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04d_prof_bench.err; final=$rc; }
head -40 gpurun_out/prof4/run_kernel_stats.csv | cut -d, -f1-8
if [ -n "${PYTEST_FILES:-}" ]; then
timeout -k 10 600 python -u -m pytest $PYTEST_FILES -m gpu -v -s --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r04d_pytest.log 2>&1
rc=$?; tail -6 gpurun_out/r04d_pytest.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || final=$rc
fi
exit $final
