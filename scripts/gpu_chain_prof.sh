cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "chain or arith or ray_wave or tilt or raywave or kb or full" > gpurun_out/pytest_chain.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
AB_WAVES=4 PYTEST_K=none bash scripts/gpu_chain_ab.sh || exit $?
rm -rf gpurun_out/pmc_* gpurun_out/prof
bash scripts/gpu_profile.sh
