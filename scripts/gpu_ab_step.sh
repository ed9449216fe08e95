#!/bin/bash
# A/B of whole-step builds: the griddata / faithful GPU tests on the in-tree library, then the
# default bench (shortened: no CPU baseline, no extras) for each library named in LIBS, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-faithful or griddata or cone or patch}" > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in ${LIBS:-hip base}; do
    AKB_LIB=$PWD/akbraytracing_amd/lib/libakb_$v.so timeout -k 10 300 python bench.py --steps 60 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/ab_${v}_$k.json 2> gpurun_out/ab_${v}_$k.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}_$k.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d.get('ms_per_step_no_ramp') or 0,4))"
  done
done
