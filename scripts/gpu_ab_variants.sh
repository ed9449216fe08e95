#!/bin/bash
# Interleaved A/B of whole default steps over variants "lib|ENV=V ...|bench args" (';'-separated
# in VARIANTS), ROUNDS rounds; one summary line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-hip||}"
for k in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i + 1))
    IFS='|' read -r lib envs args <<< "$v"
    lib=$(echo $lib)
    env AKB_LIB=$PWD/akbraytracing_amd/lib/libakb_$lib.so $envs timeout -k 10 300 python bench.py --steps 60 --warmup 30 --no-cpu-baseline --no-extras $args > gpurun_out/abv_${i}_$k.json 2> gpurun_out/abv_${i}_$k.err || { tail -5 gpurun_out/abv_${i}_$k.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abv_${i}_$k.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],4), round(d.get('ms_per_step_no_ramp') or 0,4), 'chain', round(d.get('faithful_chain_ms') or 0,4))" "$v"
  done
done
