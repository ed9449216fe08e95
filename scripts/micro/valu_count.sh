#!/bin/bash
# PMC passes over scripts/micro/valu_count (counter calibration), one counter group per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for SET in "SQ_INSTS_VALU SQ_WAVES" "SQ_INSTS_VALU_TRANS_F64" "SQ_INSTS_VALU_FMA_F64" "SQ_INSTS_VALU_MUL_F64" "SQ_INSTS_VALU_ADD_F64" "SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/vc_$i -o run -- scripts/micro/valu_count > gpurun_out/vc_$i.log 2>&1
  rc=$?; echo "set $i ($SET) exit $rc"; [ $rc -eq 0 ] || exit $rc
done
