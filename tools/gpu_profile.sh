#!/bin/bash
# Bench + rocprofv3 evidence for profiles/: the bench line, then a kernel-trace/stats pass and
# one PMC pass per counter (FETCH_SIZE, WRITE_SIZE) on the dominant kernel, all on
# `bench.py --profile-only` (the serial HIP-event pass the roofline figures come from), never
# combining counters with tracing.  Summary -> gpurun_out/prof/pmc_summary.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
K=${KREGEX:-k_cc_step_pk}
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "$O/$name.log"; [ $rc -eq 0 ] || exit $rc; }
if [ -z "${SKIP_BENCH:-}" ]; then
  run bench 600 python bench.py ${BENCH_ARGS:-}
  grep '^{' $O/bench.log > $O/bench.json || true
  if [ -z "${SKIP_PROF_ONLY:-}" ]; then
    run prof_only 300 python bench.py --profile-only ${BENCH_ARGS:-}
    grep '^{' $O/prof_only.log > $O/prof_only.json || true
  fi
fi
[ -z "${SKIP_KT:-}" ] && run kt ${STEP_SECS:-600} rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --profile-only ${PROF_ARGS---lean-pass-only} ${BENCH_ARGS:-}
[ -n "${SKIP_PMC:-}" ] && exit 0
run fetch ${STEP_SECS:-600} rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/fetch -o run --output-format csv -- python3 bench.py --profile-only ${PROF_ARGS---lean-pass-only} ${BENCH_ARGS:-}
run write ${STEP_SECS:-600} rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/write -o run --output-format csv -- python3 bench.py --profile-only ${PROF_ARGS---lean-pass-only} ${BENCH_ARGS:-}
python3 - "$K" <<'PY'
import csv, glob, json, sys
k = sys.argv[1]
out = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    by = {}  # per template instantiation: the lean and the profiling superstep differ
    for f in glob.glob(f"gpurun_out/prof/{ctr.split('_')[0].lower()}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == ctr and k in r.get("Kernel_Name", ""):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                vals, durs = by.setdefault(name, ([], []))
                vals.append(float(r["Counter_Value"]))
                try:
                    durs.append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
                except (KeyError, ValueError):
                    pass
    if by:
        # the lean instantiations (PROF, the second template flag, false: no work counters) the timed
        # run launches — k_cc_step_pk has a long- and a short-window form since round 5; their
        # launches are pooled (the per-launch figure is over every superstep of the query)
        def prof_flag(n):
            a = n[n.find("<") + 1:n.rfind(">")].split(",")
            return a[1].strip() if len(a) > 1 else "false"
        lean = [n for n in by if prof_flag(n) == "false"] or list(by)
        vals = [x for n in lean for x in by[n][0]]
        durs = [x for n in lean for x in by[n][1]]
        out[ctr] = {"kernel": " + ".join(sorted(lean)), "dispatches": len(vals),
                    "mean_kb_per_dispatch": sum(vals) / len(vals), "total_kb": sum(vals),
                    "mean_dispatch_us_under_pmc": sum(durs) / len(durs) if durs else None,
                    "per_instantiation": {n: len(by[n][0]) for n in lean},
                    "other_instantiations": {n: len(v[0]) for n, v in by.items() if n not in lean}}
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["traffic_bytes_per_launch"] = {
        "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE counts "
                   "half of a wide read; narrow 4/8-B gathers are uncalibrated; Infinity-Cache hits are counted)",
        "value": 2 * out["FETCH_SIZE"]["mean_kb_per_dispatch"] * 1024 + out["WRITE_SIZE"]["mean_kb_per_dispatch"] * 1024}
json.dump(out, open("gpurun_out/prof/pmc_summary.json", "w"), indent=1)
print(json.dumps(out)[:600])
PY
find $O -name '*stats.csv' | head
