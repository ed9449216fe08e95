#!/bin/bash
# The committed profile of HEAD's bench: kernel trace + stats of the default bench command
# (gpurun_out/prof), then the PMC passes (scripts/gpu_pmc.sh) over a short bench run; summarise
# with  python scripts/summarize_profiles.py <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py ${PROFILE_BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?; echo "stats run exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_bench.err; exit $rc; }
PMC_CMD="${PMC_CMD:-python3 bench.py --steps 5 --warmup 3 --ramp-ms 0 --no-cpu-baseline --no-extras}" bash scripts/gpu_pmc.sh
