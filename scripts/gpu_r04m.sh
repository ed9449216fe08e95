#!/bin/bash
# Round-4 GPU pass 13: the pipelined patch kernel's stage split S (sweeps 1..S in stage 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 4 5 6 7 8; do
  AKB_GD_PATCH_S=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof13_$S -o run -- \
      python3 scripts/micro_faithful.py --reps 6 --out /tmp/mf_$S.npz > gpurun_out/r04m_$S.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  echo "S=$S $(grep k_gd_cone_patch gpurun_out/prof13_$S/run_kernel_stats.csv | cut -d, -f1-5)"
  rm -f gpurun_out/prof13_$S/run_kernel_trace.csv
done
python3 -c "
import numpy as np
a = np.load('/tmp/mf_6.npz')
for S in (4, 5, 7, 8):
    b = np.load(f'/tmp/mf_{S}.npz')
    print(S, {k: bool(np.array_equal(a[k], b[k], equal_nan=True)) for k in a.files})"
