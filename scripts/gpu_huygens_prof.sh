#!/bin/bash
# Kernel trace + PMC passes of the Huygens stage (scripts/bench_huygens.py: 1e7 sources -> 65^2
# targets), one counter group per rocprofv3 run; outputs under gpurun_out/ for
# scripts/summarize_huygens.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 scripts/bench_huygens.py --reps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hprof -o run -- $CMD \
    > gpurun_out/hprof.log 2>&1
rc=$?; echo "kernel trace exit $rc"; [ $rc -eq 0 ] || exit $rc
i=0
for SET in "SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES" "SQ_INSTS_VALU_FMA_F64" "SQ_INSTS_VALU_MUL_F64" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_INT32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "k_huygens\\(" --output-format csv \
      -d gpurun_out/hpmc_$i -o run -- python3 scripts/bench_huygens.py --reps 1 > gpurun_out/hpmc_$i.log 2>&1
  rc=$?; echo "pmc set $i ($SET) exit $rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
