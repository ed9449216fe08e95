#!/bin/bash
# One gpurun call per kernel iteration: the GPU tests (not the slow ones), then three short bench
# runs (40 steps, no extras); every step under its own time limit, a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_iter.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_iter.log | head -20; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 30 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} \
      > gpurun_out/it_$i.json 2> gpurun_out/it_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/it_$i.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/it_$i.json'));print('ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4))"
done
exit 0
