#!/bin/bash
# PSF transform parity tests, then psf_stack timings at the bench's and the example's sizes (line
# transforms, then the column-pass path for A/B - or, with BASE=<another build of the library>,
# the in-tree library against that build, alternating), then the same under rocprofv3 --kernel-trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${PYTEST_K:-psf}" > gpurun_out/pytest_psf.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_psf.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$BASE" ]; then
  for k in 1 2; do
    echo "in-tree"; timeout -k 10 120 python -u scripts/micro_psf_cols.py || exit $?
    echo "base"; AKB_LIB=$PWD/$BASE timeout -k 10 120 python -u scripts/micro_psf_cols.py || exit $?
  done
else
  timeout -k 10 120 python -u scripts/micro_psf_cols.py || exit $?
  AKB_PSF_PATH=cols timeout -k 10 120 python -u scripts/micro_psf_cols.py || exit $?
fi
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_psf" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/micro_psf_cols.py" > "$GRAFT_REPO_ROOT/gpurun_out/psf_prof.log" 2>&1
rc=$?; echo "rocprof exit $rc"; exit $rc
