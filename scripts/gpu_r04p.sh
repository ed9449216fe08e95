#!/bin/bash
# Round-4 GPU pass 15: the back stream's priority (the faithful chain is now the step's critical
# stream; its small kernels wait for CUs behind the passes), interleaved bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for pr in 0 -1; do
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-extras --back-priority=$pr \
        > gpurun_out/r04p_${pr}_$rep.json 2> gpurun_out/r04p_${pr}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04p_${pr}_$rep.err; exit $rc; }
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/r04p_${pr}_$rep.json') if l.startswith('{')][-1])
print('prio $pr', $rep, round(d['ms_per_step'], 4), round(d['value'] / 1e10, 3), round(d['faithful_finish_ms'], 3))"
  done
done
