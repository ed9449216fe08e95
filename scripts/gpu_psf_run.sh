cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PYTEST_K=psf VARIANTS="env:AKB_PSF_PEAK=f64 env:AKB_PSF_PEAK=f32" bash scripts/gpu_psf_ab.sh || exit $?
timeout -k 10 300 python -u scripts/bench_psf_example.py --out gpurun_out/psf_example.json > gpurun_out/psf_example.log 2>&1; rc=$?; tail -12 gpurun_out/psf_example.log; exit $rc
