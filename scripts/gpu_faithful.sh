#!/bin/bash
# Stage times and kernel trace of the faithful PSF chain (griddata -> plane correction -> psf_calc)
# on the C3 trace's own hits: optional GPU tests (PYTEST_K), scripts/bench_faithful.py, then the
# same under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_faithful.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_faithful.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u scripts/bench_faithful.py --reps 3 ${FAITHFUL_ARGS:-} > gpurun_out/faithful.log 2>&1
rc=$?; tail -40 gpurun_out/faithful.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_faithful" -o run -- \
    python3 "$GRAFT_REPO_ROOT/scripts/bench_faithful.py" --reps 2 > "$GRAFT_REPO_ROOT/gpurun_out/faithful_prof.log" 2>&1
rc=$?; echo "rocprof exit $rc"; exit $rc
