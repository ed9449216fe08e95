#!/bin/bash
# Interleaved bench runs of library / environment variants: VARIANTS is a list of
# "<lib-tag or default>:<VAR=value,...>" (lib tag: akbraytracing_amd/lib/ab_<tag>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
  for v in $VARIANTS; do
    lib=${v%%:*}; envs=${v#*:}; envs=${envs//,/ }
    libenv=""; [ "$lib" != "default" ] && libenv="AKB_LIB=$PWD/akbraytracing_amd/lib/ab_$lib.so"
    env $libenv $envs timeout -k 10 200 python bench.py --steps ${STEPS:-100} --warmup 30 --no-cpu-baseline --no-extras \
        > gpurun_out/var.json 2> gpurun_out/var.err || { tail -5 gpurun_out/var.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/var.json').read().strip().splitlines()[-1]);print('$v', 'ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4))"
  done
done
