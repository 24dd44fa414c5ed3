#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE; separate passes, no tracing) of the CC superstep kernel on
# the C4-shaped 100M-update graph, next to its algorithmic bytes.  Summary -> gpurun_out/c4pmc/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4pmc; mkdir -p $O
A="--config c4 --c4-interactions ${C4I:-33333334} --c4-users ${C4U:-5000000}"
timeout -k 10 300 python3 bench.py $A > $O/bench.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex k_cc_step_pk -d $O/$c -o run --output-format csv -- python3 bench.py $A > $O/$c.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, json
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"gpurun_out/c4pmc/{c}/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if r.get("Counter_Name") == c]
    out[c] = {"dispatches": len(v), "mean_kb": sum(v) / max(1, len(v))}
b = [json.loads(l) for l in open("gpurun_out/c4pmc/bench.log") if l.startswith("{")][-1]
out["bench"] = b["kernels"]["cc_step"]
out["traffic_bytes_per_launch"] = 2 * out["FETCH_SIZE"]["mean_kb"] * 1024 + out["WRITE_SIZE"]["mean_kb"] * 1024
json.dump(out, open("gpurun_out/c4pmc/summary.json", "w"), indent=1)
print(json.dumps(out))
PY
