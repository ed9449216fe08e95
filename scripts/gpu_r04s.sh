#!/bin/bash
# Round-4 GPU pass 16: the pipelined patch kernel on fewer than all CUs (the rest left to the other
# streams' kernels), interleaved bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for gsz in 256 224 192; do
    AKB_GD_PATCH_GRID=$gsz timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-extras \
        > gpurun_out/r04s_${gsz}_$rep.json 2> gpurun_out/r04s_${gsz}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04s_${gsz}_$rep.err; exit $rc; }
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/r04s_${gsz}_$rep.json') if l.startswith('{')][-1])
print('grid $gsz', $rep, round(d['ms_per_step'], 4), round(d['value'] / 1e10, 3), round(d['faithful_finish_ms'], 3))"
  done
done
