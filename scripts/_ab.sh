cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_all.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err; rc=$?; cat gpurun_out/bench_full.json; tail -3 gpurun_out/bench_full.err; exit $rc
