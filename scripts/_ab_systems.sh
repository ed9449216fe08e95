cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in "" 1 "" 1; do
  AKB_BENCH_NO_KEVENTS=$v timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('noev=$v ms/step', round(d['ms_per_step'],4), 'pass2', round(d['pass2_kernel_ms'],4))"
done
