#!/bin/bash
# Round-4 GPU pass 14: the faithful begin (cell pass) on the back stream vs RayWave's finish / copy
# streams, interleaved bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for bsm in back fin copy; do
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-extras --begin-stream $bsm \
        > gpurun_out/r04o_${bsm}_$rep.json 2> gpurun_out/r04o_${bsm}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04o_${bsm}_$rep.err; exit $rc; }
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/r04o_${bsm}_$rep.json') if l.startswith('{')][-1])
print('$bsm', $rep, round(d['ms_per_step'], 4), round(d['value'] / 1e10, 3))"
  done
done
