#!/bin/bash
# Instruction-mix / wait counters (SQ_*, one group per pass, no tracing) of the C4 1B headline's
# serial lean pass (bench.py --profile-only --lean-pass-only), for the kernels in $KREGEX.
# Summary -> gpurun_out/c4sq/summary.txt (per kernel: counter totals and per-dispatch means).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4sq${SQ_TAG:-}; mkdir -p $O
K=${KREGEX:-k_cc_step_pk}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 540 rocprofv3 --pmc $grp --kernel-include-regex "$K" -d $O/p$i -o run --output-format csv -- \
    python3 bench.py --profile-only --lean-pass-only --no-cpu-baseline --no-secondary > $O/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p$i.log; exit $rc; }
done
python3 - "$O" <<'PY' | tee $O/summary.txt
import csv, glob, collections, json, sys
O = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
per = collections.defaultdict(dict)  # (pass, dispatch order) -> counter values
for f in sorted(glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True)):
    pas = f[len(O) + 1:].split("/")[0]
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
        per[(pas, k[0], int(r.get("Dispatch_Id", 0) or 0))][r["Counter_Name"]] = float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k[0][:56]:56s} {k[1]:28s} total {tot[k]:.4g}  per-dispatch {tot[k]/n[k]:.4g}  dispatches {n[k]}")
with open(O + "/per_dispatch.jsonl", "w") as o:
    for key in sorted(per):
        o.write(json.dumps({"pass": key[0], "kernel": key[1], "dispatch": key[2], **per[key]}) + "\n")
PY
