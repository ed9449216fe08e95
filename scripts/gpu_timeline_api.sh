#!/bin/bash
# rocprofv3 kernel + HIP runtime API trace of a 30-step bench (no extras): where the host waits
# relative to the kernels (scripts/step_timeline.py --api)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/tla -o run -- \
    python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/tla.log 2>&1
echo "rc $?"
