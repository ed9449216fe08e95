#!/bin/bash
# The faithful chain alone (scripts/micro_faithful.py on the C3 trace's hits): kernel trace + stats,
# then one PMC pass per counter group over the cone solve's kernels (k_gd_*), for
# scripts/summarize_profiles.py TAG -> profiles/TAG_faithful_roofline.json and the stats csv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 scripts/micro_faithful.py --reps 10 > gpurun_out/prof_faithful.log 2>&1
rc=$?; echo "kernel trace exit $rc"; [ $rc -eq 0 ] || exit $rc
PMC_REGEX="k_gd_" PMC_CMD="python3 scripts/micro_faithful.py --reps 3" \
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU_FMA_F64;SQ_INSTS_VALU_MUL_F64;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64;GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU;SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
    bash scripts/gpu_pmc.sh
