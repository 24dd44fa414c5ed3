#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench.  Every GPU step has its own time
# limit; a fault/abort/timeout (rc >= 124 or signal) ends the script.  Test *failures*
# (pytest rc 1) do not, so the bench still reports.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m1 -o 'gfx9[0-9a-z]*' > gpurun_out/arch.txt
for s in ${STEPS:-pytest smoke bench}; do
  case $s in
    pytest) step pytest_gpu ${PYTEST_SECS:-900} python -u -m pytest tests -m "${PYTEST_MARK:-gpu}" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke)  step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
    bench)  step bench ${BENCH_SECS:-900} python -u bench.py ${BENCH_ARGS:-} ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
