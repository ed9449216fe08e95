#!/bin/bash
# Round-4 GPU pass 10: the pipelined patch kernel's per-phase cycles (the top wait split into this
# wave's own outstanding memory and the barrier).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AKB_GD_PATCH_CLOCK=1 timeout -k 10 300 python3 scripts/micro_faithful.py --reps 2 > gpurun_out/r04j_clk.log 2>&1
rc=$?; grep AKB_GD_PATCH_CLOCK gpurun_out/r04j_clk.log | tail -1; exit $rc
