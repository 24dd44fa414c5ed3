#!/bin/bash
# Per-dispatch kernel trace of the serial profiled pass (bench.py --profile-only) for
# step-by-step duration analysis; every step time-limited, first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/trace; mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "$O/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run c2_kt 300 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 bench.py --profile-only ${BENCH_ARGS:-}
if [ -n "${C4ARGS:-}" ]; then
  run c4 600 python3 bench.py --config c4 $C4ARGS
fi
