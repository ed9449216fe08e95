#!/bin/bash
# A/B of an environment knob by per-kernel rocprofv3 stats over a short bench run:
#   bash scripts/ab_env.sh VAR "v1 v2 ..." KERNEL_REGEX
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VAR=$1; VALS=$2; RE=$3
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit $?
  python3 - "$v" "$RE" <<'PY'
import csv, json, sys
v, rx = sys.argv[1], sys.argv[2]
import re
rows = list(csv.DictReader(open(f"gpurun_out/ab_{v}/run_kernel_stats.csv")))
b = json.loads(open(f"gpurun_out/ab_{v}.json").read())
out = {r["Name"][:40]: round(float(r["AverageNs"]) / 1e3, 1) for r in rows if re.search(rx, r["Name"])}
print(v, round(b["ms_per_step"], 4), out, flush=True)
PY
done
