#!/bin/bash
# Round-end rehearsal in one gpurun call: the GPU suite, smoke(), the default bench line, then the
# committed profile of that bench (scripts/gpu_profile.sh: kernel trace + PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
bash scripts/gpu_profile.sh
