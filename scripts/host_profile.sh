#!/bin/bash
# Where the host's time per bench step goes: bench.py under cProfile (200 steps), the top
# functions by own time and by cumulative time into gpurun_out/host_prof.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/host.prof bench.py --steps 200 --warmup 5 --no-cpu-baseline \
    --no-extras > gpurun_out/host_bench.json 2> gpurun_out/host_bench.err || { tail -5 gpurun_out/host_bench.err; exit 1; }
python - <<'PY' > gpurun_out/host_prof.txt
import pstats
s = pstats.Stats("gpurun_out/host.prof")
s.sort_stats("tottime").print_stats(45)
s.sort_stats("cumulative").print_stats(60)
PY
head -c 300 gpurun_out/host_bench.json
