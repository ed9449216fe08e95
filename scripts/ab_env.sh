#!/bin/bash
# A/B of one environment variable over interleaved bench runs:
#   bash scripts/ab_env.sh VAR "valA valB" [steps] [warmup]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
var=$1; vals=$2; steps=${3:-200}; warm=${4:-30}
for rep in 1 2; do
  for v in $vals; do
    env "$var=$v" timeout -k 10 200 python bench.py --steps $steps --warmup $warm --no-cpu-baseline --no-extras \
        > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$var=$v ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4), 'host', round(d['host_issue_ms_per_step'],4))"
  done
done
