#!/bin/bash
# Round-4 GPU pass 2: cone solve, the one-workgroup pupil post, the pipelined faithful PSF.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_faithful_gpu.py} -m gpu -x -v -s --timeout 300 \
  --timeout-method thread -k "${PYTEST_K:-cone or pupil_post or gd_axes or faithful or nonuniform or flagged or nan_source or two_streams}" \
  > gpurun_out/r04b_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r04b_pytest.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 300 python -u bench.py $BENCH_ARGS > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err
  rc=$?; tail -c 3000 gpurun_out/r04b_bench.json; [ $rc -eq 0 ] || exit $rc
fi
