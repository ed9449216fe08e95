#!/bin/bash
# Round-4 GPU pass 5: the faithful chain's kernels reworked (register-resident cone patches, one
# launch per band sweep, the pupil post's prefilter in LDS): parity tests, then the bench under a
# kernel trace and plain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
timeout -k 10 700 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_faithful_gpu.py tests/test_faithful_dist_gpu.py tests/test_fullsize_gpu.py} \
  -m gpu -x -v -s --timeout 300 --timeout-method thread -k "${PYTEST_K:-cone or gradient or pupil_post or faithful or griddata or psf_calc or wave_maps or sharded}" \
  > gpurun_out/r04e_pytest.log 2>&1
rc=$?; tail -8 gpurun_out/r04e_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --ramp-ms 0 --no-ramp-form \
    > gpurun_out/r04e_prof_bench.json 2> gpurun_out/r04e_prof_bench.err
rc=$?; echo "prof exit $rc"; fatal $rc && exit $rc
head -24 gpurun_out/prof5/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline} > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err
rc=$?; tail -c 1500 gpurun_out/r04e_bench.json; exit $rc
