#!/bin/bash
# The driver's bench form (20 steps after 5 warm-up) at several clock-ramp lengths, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for r in ${RAMPS:-300 1000}; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ramp-ms $r --no-cpu-baseline --no-extras > gpurun_out/rl.json 2> gpurun_out/rl.err || { tail -5 gpurun_out/rl.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rl.json').read().strip().splitlines()[-1]);print('ramp $r', round(d['ms_per_step'],4), d['clock_ramp'])"
  done
done
