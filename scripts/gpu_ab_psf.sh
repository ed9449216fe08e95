#!/bin/bash
# A/B of the default step between the in-tree library and libakb_base.so (LIBS), after the PSF GPU
# tests: step, chain and the PSF's in-step and alone times per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-psf}" > gpurun_out/pytest_psf.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_psf.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in ${LIBS:-hip base}; do
    AKB_LIB=$PWD/akbraytracing_amd/lib/libakb_$v.so timeout -k 10 300 python bench.py --steps 60 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/abp_${v}_$k.json 2> gpurun_out/abp_${v}_$k.err || { tail -5 gpurun_out/abp_${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abp_${v}_$k.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d.get('ms_per_step_no_ramp') or 0,4), 'chain', round(d.get('faithful_chain_ms') or 0,4), 'psf', round(d.get('psf_ms') or 0,4), 'alone', round(d.get('psf_alone_ms') or 0,4), round(d.get('psf_device_ms') or 0,4))"
  done
done
