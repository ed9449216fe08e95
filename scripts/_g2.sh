cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pipeline or ray_wave_65" > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
for F in 2 1 2 1; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --fuse $F > gpurun_out/b_$F.json 2>gpurun_out/b.err; rc=$?; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/b_$F.json'));print('fuse', $F, round(d['ms_per_step'],4), round(d['pass2_kernel_ms'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof2.log 2>&1; echo prof $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -2 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
