#!/bin/bash
# Round 6: the C4 1B query at N = 1 with and without the window-class hybrid (--hybrid-n1: week, day, hour
# on a time-slice replica), same box, back to back; the checks (840 views' summed fields, superstep sum
# included) must be equal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-n1hyb_r6}
A="--no-cpu-baseline --no-secondary --no-edge-counts --steps ${STEPS:-5} --warmup 1"
timeout -k 10 420 python -u bench.py $A --hybrid "" > gpurun_out/${T}_base.json 2> gpurun_out/${T}_base.err || { tail -5 gpurun_out/${T}_base.err; exit 1; }
timeout -k 10 420 python -u bench.py $A --hybrid ${HYB:-mwdh} > gpurun_out/${T}_hyb.json 2> gpurun_out/${T}_hyb.err || { tail -5 gpurun_out/${T}_hyb.err; exit 1; }
python3 - gpurun_out/${T}_base.json gpurun_out/${T}_hyb.json <<'PY'
import json, sys
a, b = (json.loads([l for l in open(f) if l.startswith("{")][-1]) for f in sys.argv[1:3])
for x in (a, b):
    print(x["ms_per_step"], x["value"], x["check"], x["config"]["parallelism"])
assert a["check"] == b["check"], "checks differ"
print("checks equal")
PY
