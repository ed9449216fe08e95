#!/bin/bash
# The bench's N > 1 path rehearsed on one GPU (two ranks sharing it over gloo: every line of the
# multi-rank code runs, the RCCL transport aside), then the C2 configuration's line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AKB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu-baseline \
    > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err
rc=$?; echo "n2 gloo exit $rc"; tail -c 1500 gpurun_out/bench_n2_gloo.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_n2_gloo.err; exit $rc; }
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; echo "c2 exit $rc"; tail -c 800 gpurun_out/bench_c2.json; exit $rc
