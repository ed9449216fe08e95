#!/bin/bash
# Round-4 final pass, part 1: the whole GPU suite, smoke(), the default bench line, and configs[3]
# sharded over 8 gloo ranks (tests/test_c4_gpu.py is part of the suite).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 600 --timeout-method thread > gpurun_out/r04k_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04k_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04k_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r04k_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04k_bench.err; exit $rc; }
python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/r04k_bench.json') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('value', 'ms_per_step', 'ms_per_step_no_ramp', 'faithful_chain_ms', 'faithful_finish_ms', 'psf_ms', 'faithful_pipelined_single_ms', 'faithful_psf_chain_ms')})
print('cpu_baseline', d.get('cpu_baseline'))"
