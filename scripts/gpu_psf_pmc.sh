#!/bin/bash
# PMC passes over the PSF line kernels (scripts/micro_psf_cols.py: 2048^2 and 16384^2), one
# counter group per rocprofv3 run, outputs under gpurun_out/psfpmc_<i>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for SET in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32" \
           ${PMC_EXTRA:-}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $SET --kernel-include-regex "k_psf_line" --output-format csv \
      -d gpurun_out/psfpmc_$i -o run -- python3 scripts/micro_psf_cols.py --reps 2 > gpurun_out/psfpmc_$i.log 2>&1
  rc=$?; echo "pmc set $i ($SET) exit $rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
