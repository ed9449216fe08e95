#!/bin/bash
# Is the short-run bench slower because of the device clock? The driver's 20 / 5 steps with and
# without a clock ramp ahead of the warm-up, against 20 / 30 and 100 / 30.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --ramp-ms 300" "--steps 20 --warmup 30" "--steps 100 --warmup 30" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --ramp-ms 300"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-extras > gpurun_out/ramp_$i.json 2> gpurun_out/ramp_$i.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ramp_$i.err; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/ramp_$i.json').read().strip().splitlines()[-1]);print('$a', '->', round(d['ms_per_step'],4), d['clock_ramp'])"
done
