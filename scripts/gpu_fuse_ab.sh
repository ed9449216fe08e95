#!/bin/bash
# A/B of the pass-1 fusion in the whole step: bench.py --fuse 2 (pass 1 carries
# run k-2's tilt and run k-3's OPD), --fuse 1 (the tilt only; the OPD on the back stream) and
# --fuse 0 (pass 1 alone; tilt + OPD as k_tilt_opd_sink on the back stream), alternating, each in
# the default form and the driver's 20 / 5 form (ms_per_step_no_ramp).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in ${ROUNDS:-1 2}; do
  for f in ${MODES:-2 1 0}; do
    timeout -k 10 300 python bench.py --fuse $f --steps ${STEPS:-60} --warmup ${WARMUP:-30} --no-cpu-baseline --no-extras \
      > gpurun_out/fuse_${f}_$k.json 2> gpurun_out/fuse_${f}_$k.err || { tail -5 gpurun_out/fuse_${f}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/fuse_${f}_$k.json').read().strip().splitlines()[-1]); print('fuse $f', round(d['ms_per_step'],4), round(d.get('ms_per_step_no_ramp') or 0,4), 'chain', round(d.get('faithful_chain_ms') or 0,4), 'pass2', round(d['pass2_kernel_ms'],4))"
  done
done
