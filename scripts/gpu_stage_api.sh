#!/bin/bash
# The stage API block of bench.py (per-primitive GB/s on the bench's 1e7-ray rows), per library
# variant (LIBS: tags of akbraytracing_amd/lib/ab_<tag>.so; "default" = the in-tree build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  libenv=""; [ "$lib" != "default" ] && libenv="AKB_LIB=$PWD/akbraytracing_amd/lib/ab_$lib.so"
  env $libenv timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/stage_$lib.json 2> gpurun_out/stage_$lib.err
  rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/stage_$lib.err; exit $rc; }
  python -c "
import json;d=json.loads(open('gpurun_out/stage_$lib.json').read().strip().splitlines()[-1])['stage_api']
print('$lib', {k: round(v.get('frac_of_hbm', v.get('gbs', 0)), 3) for k, v in d.items() if isinstance(v, dict)})"
done
