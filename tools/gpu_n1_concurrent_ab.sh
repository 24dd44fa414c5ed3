#!/bin/bash
# Round 6: the C4 1B query at N = 1 with the hybrid, the graph's and the replica's runs one after the
# other (--hybrid-serial) vs on two host threads (default), back to back on one box; checks must be equal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-n1conc_r6}
A="--no-cpu-baseline --no-secondary --no-edge-counts --steps ${STEPS:-5} --warmup 1"
timeout -k 10 420 python -u bench.py $A --hybrid-serial > gpurun_out/${T}_serial.json 2> gpurun_out/${T}_serial.err || { tail -5 gpurun_out/${T}_serial.err; exit 1; }
timeout -k 10 420 python -u bench.py $A > gpurun_out/${T}_conc.json 2> gpurun_out/${T}_conc.err || { tail -5 gpurun_out/${T}_conc.err; exit 1; }
python3 - gpurun_out/${T}_serial.json gpurun_out/${T}_conc.json <<'PY'
import json, sys
a, b = (json.loads([l for l in open(f) if l.startswith("{")][-1]) for f in sys.argv[1:3])
for x in (a, b):
    print(x["ms_per_step"], x["value"], x["check"])
assert a["check"] == b["check"], "checks differ"
print("checks equal")
PY
