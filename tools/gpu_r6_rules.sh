#!/bin/bash
# Round 6: the hub size rules for every graph (rgpu.cpp hub_threshold, hub_pro) — replica A/B on the
# 1B week slice (21 hops x {w,d,h}, P = 8 blocks), then the full GPU suite + smoke on this build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-rules_r6}
timeout -k 10 420 python -u tools/part_sim.py --interactions 333333334 --parts 8 --probe-rounds 0 --profile-rounds 1 \
  --hybrid wdh --replica-only --replica-ab "RGPU_HEAVY=512;RGPU_HEAVY=1024;RGPU_HUB_PRO=32" \
  > gpurun_out/part_$T.jsonl 2> gpurun_out/part_$T.err || { tail -5 gpurun_out/part_$T.err; exit 1; }
cut -c1-400 gpurun_out/part_$T.jsonl
TAG=$T bash tools/gpu_suite_r6.sh
