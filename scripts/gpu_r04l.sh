#!/bin/bash
# Round-4 GPU pass 12: the faithful chain's kernel trace in order (which copies sit in a finish).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof12 -o run -- \
    python3 scripts/micro_faithful.py --reps 3 > gpurun_out/r04l_micro.log 2>&1
rc=$?; tail -1 gpurun_out/r04l_micro.log; exit $rc
