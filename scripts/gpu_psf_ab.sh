#!/bin/bash
# A/B of the PSF transforms: optional parity tests (PYTEST_K), then a kernel trace of
# scripts/micro_psf_cols.py per variant. VARIANTS: "default", "lib:<name>" (AKB_LIB =
# akbraytracing_amd/lib/ab_<name>.so) or "env:<VAR>=<value>".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_psf.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_psf.log; [ $rc -eq 0 ] || exit $rc
fi
n=0
for v in default ${VARIANTS:-}; do
  n=$((n+1))
  case "$v" in
    lib:*) envs="AKB_LIB=$GRAFT_REPO_ROOT/akbraytracing_amd/lib/ab_${v#lib:}.so" ;;
    env:*) envs="${v#env:}" ;;
    *) envs="" ;;
  esac
  (cd /tmp && env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/psfab_$n" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/micro_psf_cols.py" > "$GRAFT_REPO_ROOT/gpurun_out/psfab_$n.log" 2>&1)
  rc=$?; echo "variant $n ($v) exit $rc"; grep pupil gpurun_out/psfab_$n.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
