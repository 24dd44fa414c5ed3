#!/bin/bash
# Live-ingest evidence: the live / RGEV parity tests, then the C5 bench with host phase times
# (RGPU_HOSTPROF=1).  STEPS="full" runs the whole GPU suite instead of the live subset.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/c5
T=${TESTS:-tests/test_gpu_live.py tests/test_gpu_rgev.py}
timeout -k 10 600 python3 -m pytest $T -m gpu -x -q > gpurun_out/c5/pytest_live.log 2>&1 || { tail -30 gpurun_out/c5/pytest_live.log; exit 1; }
tail -2 gpurun_out/c5/pytest_live.log
RGPU_HOSTPROF=1 timeout -k 10 600 python3 -u bench.py --config c5 ${C5ARGS:-} > gpurun_out/c5/c5.log 2>&1; rc=$?
grep -v "^\[rgpu seal_delta\]\|hostprof\|pack_delta\]\|finish_delta\]" gpurun_out/c5/c5.log | tail -9; exit $rc
