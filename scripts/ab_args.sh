#!/bin/bash
# A/B of bench.py argument sets over interleaved runs:  bash scripts/ab_args.sh "ARGS_A" "ARGS_B" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for rep in 1 2; do
  for a in "$@"; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-cpu-baseline --no-extras $a \
        > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('[$a] ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4), 'psf', round(d['psf_ms'],4))"
  done
done
