#!/bin/bash
# The driver's short form (--steps 20 --warmup 5) with --step-log, over bench-argument variants
# (';'-separated in VARIANTS): per step, when its main- and back-stream work completed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-}"
[ ${#VS[@]} -eq 0 ] && VS=("")
i=0
for v in "${VS[@]}"; do
  i=$((i + 1))
  timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --step-log --no-cpu-baseline --no-extras $v > gpurun_out/sl_$i.json 2> gpurun_out/sl_$i.err || { tail -5 gpurun_out/sl_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sl_$i.json').read().strip().splitlines()[-1]); s=d['step_log']['steps']; m=[r[0] for r in s]; print(repr(sys.argv[1]), round(d['ms_per_step'],4), round(d['ms_per_step_no_ramp'] or 0,4), [round(b-a,2) for a,b in zip([0]+m,m)])" "$v"
done
