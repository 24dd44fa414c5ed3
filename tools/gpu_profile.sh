#!/bin/bash
# Bench + rocprofv3 evidence for profiles/: kernel-trace/stats pass, then one PMC pass per
# counter (FETCH_SIZE, WRITE_SIZE) on the dominant kernel — never combined with tracing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "$O/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run bench 600 python bench.py ${BENCH_ARGS:-}
grep '^{' $O/bench.log > $O/bench.json || true
run kt 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
run fetch 900 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cc_step -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass
run write 900 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cc_step -d $O/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass
find $O -name '*.csv' | head -20
