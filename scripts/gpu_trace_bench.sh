#!/bin/bash
# Kernel trace + stats of a short default-form bench (no extras): per-kernel in-step durations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/tprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof -o run -- \
    python3 bench.py --steps ${STEPS:-60} --warmup 30 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/tprof_bench.json 2> gpurun_out/tprof_bench.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tprof_bench.err; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/tprof_bench.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'])"
