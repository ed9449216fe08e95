#!/bin/bash
# PMC passes (one counter group per run, kernel trace only, no sys/runtime trace) over a short
# bench run, for the roofline's HBM traffic and the FP64 instruction mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
rc=$?; echo "list exit $rc"; [ $rc -eq 0 ] || exit $rc
REGEX="${PMC_REGEX:-k_chain|k_tilt|k_opd|k_pw|k_psf|fft|k_gd|k_pupil}"
CMD="${PMC_CMD:-python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline}"
OUT="${PMC_OUT:-pmc}"
i=0
# each FP64 counter in a pass of its own (in one shared pass, r01d, FMA_F64 and MUL_F64 read
# identical; r02a measured them apart and they still agree for the pass-2 kernel: the code's mix).
# PMC_SETS="A B;C D" replaces the default list (';' between passes)
SETS="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU_FMA_F64;SQ_INSTS_VALU_MUL_F64;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64;GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU;SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU;SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
IFS=';' read -r -a SETLIST <<< "${PMC_SETS:-$SETS}"
for SET in "${SETLIST[@]}"; do
  [ -n "$SET" ] || continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$REGEX" --output-format csv \
      -d gpurun_out/${OUT}_$i -o run -- $CMD > gpurun_out/${OUT}_$i.log 2>&1
  rc=$?; echo "pmc set $i ($SET) exit $rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
exit 0
