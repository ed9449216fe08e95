#!/bin/bash
# One gpurun call: GPU tests, smoke, a short bench and a rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash / timeout / abort ends the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures, not a fault

timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" | tee -a gpurun_out/pytest_gpu.log; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc

timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc

if [ -z "${NO_PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
  rc=$?; echo "rocprof exit $rc"
fi
exit 0
