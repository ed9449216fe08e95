#!/bin/bash
# Round-4 GPU pass 9: pass 8 (persistent LDS-DMA patch kernel) then the patch / band / claim
# kernels' stall counters on the faithful chain alone (LDS waits, bank conflicts, VALU activity).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r04h.sh || exit $?
PMC_CMD="python3 scripts/micro_faithful.py --reps 2" PMC_REGEX="k_gd_cone|k_gd_claim|k_gd_cells" PMC_OUT=r04i_pmc \
PMC_SETS="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVES;SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
  bash scripts/gpu_pmc.sh
