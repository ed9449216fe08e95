#!/bin/bash
# One gpurun call for an A/B iteration: the GPU tests, then a few bench runs (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_$i.json 2> gpurun_out/b_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_$i.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/b_$i.json'));print('ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4))"
done
exit 0
