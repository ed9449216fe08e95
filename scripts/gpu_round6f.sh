#!/bin/bash
# Round-6 rehearsal on the current tree: the GPU suite, smoke(), the default bench line and the
# driver's short form, the C2 / C5 lines, the bench's kernel trace + PMC passes (scripts/gpu_profile.sh), then the
# faithful chain alone with its PMC passes (scripts/gpu_pmc_faithful.sh, outputs under pmcf_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_20_5.json 2> gpurun_out/bench_20_5.err
rc=$?; echo "bench 20/5 exit $rc"; [ $rc -eq 0 ] || exit $rc
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extras > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c exit $rc"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_profile.sh || exit $?
mkdir -p gpurun_out/bench_prof && mv gpurun_out/prof gpurun_out/pmc_* gpurun_out/bench_prof/ 2>/dev/null
bash scripts/gpu_pmc_faithful.sh
