#!/bin/bash
# Round 6: rocprofv3 evidence for profiles/ on one config (CFG=c4 default, or c2): a kernel-trace /
# stats pass, then one PMC pass per counter (FETCH_SIZE, WRITE_SIZE) over EVERY kernel of the serial
# lean profile pass (`bench.py --profile-only --lean-pass-only`: exactly the launches the bench times
# for its roofline), never combining counters with tracing.  tools/pmc_summary.py pools them per
# kernel group -> gpurun_out/prof_$CFG/pmc_summary.json (profiles/latest_pmc[_c4].json format).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-c4}
O=gpurun_out/prof_$CFG
mkdir -p $O
A="--config $CFG --profile-only --lean-pass-only ${BENCH_ARGS:-}"
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -2 "$O/$name.log"; [ $rc -eq 0 ] || exit $rc; }
[ -z "${SKIP_KT:-}" ] && run kt ${STEP_SECS:-420} rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py $A
run fetch ${STEP_SECS:-420} rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py $A
run write ${STEP_SECS:-420} rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py $A
python3 tools/pmc_summary.py $O/fetch $O/write $O/pmc_summary.json
grep '^{' $O/fetch.log > $O/prof_line.json || true
find $O/kt -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
