#!/bin/bash
# Huygens stage check: its GPU tests, then scripts/bench_huygens.py for the in-tree library and
# any variant builds named in $HUY_LIBS (AKB_LIB A/B), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "huygens or wavecalc or propagate" -v --timeout 200 --timeout-method thread > gpurun_out/huy_tests.log 2>&1
rc=$?; tail -3 gpurun_out/huy_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in "" ${HUY_LIBS:-}; do
    AKB_LIB="$lib" timeout -k 10 200 python scripts/bench_huygens.py --reps 3 > gpurun_out/huy_bench.json 2>gpurun_out/huy_bench.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/huy_bench.err; exit $rc; }
    echo "lib=${lib:-default} $(cat gpurun_out/huy_bench.json)"
  done
done
