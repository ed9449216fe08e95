#!/bin/bash
# Round-4 first GPU pass: the new parity tests (full-size PSF, qhull's triangulation, C1 at 317^2,
# non-uniform axes, the default gradient tolerance, Huygens NaN / two streams), the sweep study and
# the faithful chain's stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_fullsize_gpu.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 \
  --timeout-method thread -k "${PYTEST_K:-fullsize or ellipse or nonuniform or default_tol or flagged or nan_source or two_streams or griddata or gradient or huygens or wave_maps or psf_calc}" \
  > gpurun_out/r04a_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r04a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/study_sweeps.py > gpurun_out/r04a_sweeps.log 2>&1
rc=$?; cat gpurun_out/r04a_sweeps.log | cut -c1-3000; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_faithful.py --reps 3 > gpurun_out/r04a_faithful.log 2>&1
rc=$?; tail -8 gpurun_out/r04a_faithful.log; exit $rc
