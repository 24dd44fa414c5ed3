#!/bin/bash
# A/B of library settings on the headline bench: VARIANTS="NAME=ENV ..." (ENV as K=V,K=V).
# Each run time-limited; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
for spec in ${VARIANTS:-base=X=0}; do
  name=${spec%%=*}; envs=${spec#*=}
  echo "=== $name ($envs)"
  timeout -k 10 300 env ${envs//,/ } python3 bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-profile-pass ${BENCH_ARGS:-} > $O/$name.log 2>&1
  rc=$?; grep -o '"ms_per_step": [0-9.]*' $O/$name.log; [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
done
if [ -n "${TESTENV:-}" ]; then
  echo "=== pytest ($TESTENV)"
  timeout -k 10 600 env ${TESTENV//,/ } python3 -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; exit $rc
fi
