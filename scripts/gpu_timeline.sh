#!/bin/bash
# rocprofv3 kernel trace of a 30-step bench (no extras) for scripts/step_timeline.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- \
    python3 bench.py --steps 60 --warmup 30 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/tl.log 2>&1
echo "rc $?"
