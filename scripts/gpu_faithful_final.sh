#!/bin/bash
# The griddata / faithful GPU tests on the in-tree library, then the chain alone with its PMC passes
# (scripts/gpu_pmc_faithful.sh) for the faithful roofline of the final sources.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${PYTEST_K:-faithful or griddata or cone or patch or cells or claim}" > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_faithful.sh
