# round 6: the partitioned rehearsal (tools/part_sim.py) — PARTS, INTER (interactions of the 1B stream's
# prefix, x3 updates), TAG, PROBE (exchange-probe rounds), TRACE=1 (per-launch traces), SECS
set -u
P=${PARTS:-1,8}; I=${INTER:-100000000}; T=${TAG:-part_r6}; PR=${PROBE:-500}
mkdir -p gpurun_out
X=""; [ -n "${TRACE:-}" ] && X="--trace gpurun_out/ptrace_$T"
[ -n "${AB:-}" ] && X="$X --ab $AB"
[ -n "${HYB:-}" ] && X="$X --hybrid $HYB"
timeout -k 10 ${SECS:-1000} python -u tools/part_sim.py --interactions $I --parts $P --probe-rounds $PR --profile-rounds 1 $X > gpurun_out/$T.jsonl 2> gpurun_out/$T.err; rc=$?
tail -c 1500 gpurun_out/$T.jsonl; tail -3 gpurun_out/$T.err; exit $rc
