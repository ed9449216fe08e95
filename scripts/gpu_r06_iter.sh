#!/bin/bash
# One iteration on the box: the griddata / faithful GPU tests on the in-tree library, an A/B of the
# default step against libakb_base.so (LIBS), then the full default bench line on the in-tree library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${PYTEST_K:-faithful or griddata or cone or patch}" > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in ${LIBS:-hip base}; do
    AKB_LIB=$PWD/akbraytracing_amd/lib/libakb_$v.so timeout -k 10 300 python bench.py --steps 60 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/ab_${v}_$k.json 2> gpurun_out/ab_${v}_$k.err || { tail -5 gpurun_out/ab_${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_${v}_$k.json').read().strip().splitlines()[-1]); rf=d.get('roofline_faithful') or {}; print('$v', round(d['ms_per_step'],4), round(d.get('ms_per_step_no_ramp') or 0,4), 'chain', round(d.get('faithful_chain_ms') or 0,4), 'patch', round(rf.get('avg_ms') or 0,4))"
  done
done
[ -n "$NO_FULL" ] && exit 0
timeout -k 10 500 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_full.err; exit $rc; }
