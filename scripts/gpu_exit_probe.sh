#!/bin/bash
# Which part of the default bench leaves a crash at interpreter exit: full default run, without the
# CPU baseline, without the extras; Python's fault handler prints every thread's stack on a signal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "${@:-full|}"; do
  IFS='|' read -r name args <<< "$v"
  timeout -k 10 400 python -X faulthandler bench.py --steps 20 --warmup 10 $args > gpurun_out/exit_$name.json 2> gpurun_out/exit_$name.err
  echo "$name exit $?"
done
