# one iteration on the faithful chain: the griddata / faithful / full-size tests, a kernel trace of the
# chain alone (scripts/micro_faithful.py), the bench in the driver's 20 / 5 form. TAG=name bash scripts/gpu_iter.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "griddata or gradient or cone or gd_ or pupil_post or wave_maps or faithful or psf_calc" tests/test_faithful_gpu.py tests/test_faithful_dist_gpu.py tests/test_fullsize_gpu.py > gpurun_out/${TAG:-iter}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG:-iter}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG:-iter}_pytest.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG:-iter}_prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/micro_faithful.py --reps 20 > $GRAFT_REPO_ROOT/gpurun_out/${TAG:-iter}_micro.txt 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
tail -2 gpurun_out/${TAG:-iter}_micro.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${TAG:-iter}_bench.json 2> gpurun_out/${TAG:-iter}_bench.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/${TAG:-iter}_bench.json'))
print({k:d.get(k) for k in ['ms_per_step','ms_per_step_no_ramp','faithful_chain_ms','faithful_finish_ms','faithful_finishes_timed','psf_ms','pass2_kernel_ms']})"
