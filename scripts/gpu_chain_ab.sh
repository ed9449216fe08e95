#!/bin/bash
# The trace kernels after an arithmetic change: the GPU suite (PYTEST_K narrows it), then the bench
# at 100 / 30 steps once per pass-2 occupancy variant (AB_WAVES, default "4 6").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PYTEST_K:-}" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_chain.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
fi
for w in ${AB_WAVES:-4 6}; do
  AKB_PASS2_WAVES=$w timeout -k 10 400 python bench.py --steps 100 --warmup 30 --no-cpu-baseline > gpurun_out/bench_w$w.json 2> gpurun_out/bench_w$w.err
  rc=$?; echo "bench waves $w exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_w$w.err; exit $rc; }
  python - "$w" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_w{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], "ms_per_step", d.get("ms_per_step"), "value", d.get("value"), "pass2_kernel_ms", d.get("pass2_kernel_ms"), "psf_alone_ms", d.get("psf_alone_ms"), "roofline", d.get("roofline"))
PY
done
exit 0
