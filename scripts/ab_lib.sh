#!/bin/bash
# A/B of two builds of the library over interleaved bench runs (AKB_LIB selects the variant):
#   bash scripts/ab_lib.sh akbraytracing_amd/lib/libakb_hip_var.so [steps] [warmup]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
var=$1; steps=${2:-150}; warm=${3:-30}
for rep in 1 2; do
  for lib in "" "$var"; do
    AKB_LIB="$lib" timeout -k 10 200 python bench.py --steps $steps --warmup $warm --no-cpu-baseline --no-extras \
        > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('lib=${lib:-default} ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4))"
  done
done
