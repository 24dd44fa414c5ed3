#!/bin/bash
# Round 6: the window-class hybrid (raphtory_amd/partitioned.py) — its GPU exactness tests, bench.py's
# N > 1 path with it (2 ranks, shared-memory channel, summaries vs N = 1), then the rehearsal on the
# 1B graph (tools/part_sim.py --hybrid, P = ${PARTS:-1,8}).  Each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-hyb_r6}
timeout -k 10 300 python -u -m pytest tests/test_gpu_partitioned.py -k hybrid -x -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
[ -n "${SKIP_NRANK:-}" ] || TAG=$T N=2 SECS=300 bash tools/gpu_nrank_rehearsal_r6.sh || exit 1
RGPU_SLOTS=1 timeout -k 10 ${SECS:-800} python -u tools/part_sim.py --interactions ${INTER:-333333334} --parts ${PARTS:-1,8} \
  --probe-rounds 300 --profile-rounds 1 --hybrid ${HYB:-dh} ${REPENV:+--replica-env $REPENV} ${EXTRA:-} > gpurun_out/part_$T.jsonl 2> gpurun_out/part_$T.err; rc=$?
tail -c 1200 gpurun_out/part_$T.jsonl; tail -3 gpurun_out/part_$T.err; exit $rc
