#!/bin/bash
# PMC passes (one counter group per pass, no tracing) on the CC superstep kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ctr; mkdir -p $O
K=${KREGEX:-k_cc_step_pk}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-include-regex "$K" -d $O/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass > $O/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p$i.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/ctr/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(f"{k:32s} total {tot[k]:.4g}  per-dispatch {tot[k]/n[k]:.4g}  dispatches {n[k]}")
PY
