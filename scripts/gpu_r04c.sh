#!/bin/bash
# Round-4 GPU pass 3: the faithful / sharded-faithful / configs tests, the default bench line, and
# the bench's N > 1 path rehearsed with two gloo ranks on the one GPU (sharded faithful pupil).
# A failing test does not stop the later steps; a timeout, abort or fault ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ]; }
final=0
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests/test_faithful_gpu.py tests/test_faithful_dist_gpu.py tests/test_configs_gpu.py} \
  -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r04c_pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r04c_pytest.log; fatal $rc && exit $rc; [ $rc -eq 0 ] || final=$rc
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline} > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err
rc=$?; tail -c 2500 gpurun_out/r04c_bench.json; fatal $rc && exit $rc; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04c_bench.err; final=$rc; }
if [ -z "${NO_N2:-}" ]; then
AKB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu-baseline \
    > gpurun_out/r04c_bench_n2.json 2> gpurun_out/r04c_bench_n2.err
rc=$?; echo "n2 gloo exit $rc"; tail -c 2000 gpurun_out/r04c_bench_n2.json; fatal $rc && exit $rc; [ $rc -eq 0 ] || { tail -30 gpurun_out/r04c_bench_n2.err; final=$rc; }
fi
exit $final
