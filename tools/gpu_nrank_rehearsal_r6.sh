#!/bin/bash
# Round 6: rehearse bench.py's N > 1 path (the one the driver's 8-GPU scaling run takes) on a one-GPU
# box: torch.distributed.run with N ranks, gloo control plane, the library's shared-memory label-record
# channel instead of RCCL (RCCL refuses two ranks on one GPU), every rank on GPU 0.  It exercises the
# rank-sharded stream generation, the partitioned seal, the collective query + profile passes, the
# barrier / max-over-ranks timing and rank 0's JSON line.  The timing is NOT a scaling number (the
# ranks share one GPU).  N=${N:-2}, C4 prefix of ${INTER:-33333334} interactions (x3 updates).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-2}
INTER=${INTER:-33333334}
TAG=${TAG:-r6}
O=gpurun_out/nrank_${TAG}
timeout -k 10 ${SECS:-600} python3 bench.py --steps 2 --warmup 1 --c4-interactions $INTER --no-cpu-baseline \
  --no-secondary --no-edge-counts > ${O}_n1.json 2> ${O}_n1.err || { echo "N=1 failed"; tail -5 ${O}_n1.err; exit 1; }
timeout -k 10 ${SECS:-600} python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port ${PORT:-29517} bench.py --gpus $N --steps 2 --warmup 1 \
  --exchange shm --c4-interactions $INTER > ${O}_n$N.json 2> ${O}_n$N.err
rc=$?
echo "rc=$rc"
tail -5 ${O}_n$N.err
[ $rc -eq 0 ] || exit $rc
# the summaries' checksums must not depend on N
python3 - ${O}_n1.json ${O}_n$N.json <<'PY'
import json, sys
a, b = (json.loads([l for l in open(f) if l.startswith("{")][-1]) for f in sys.argv[1:3])
print("N=1", a["check"], a["ms_per_step"]); print("N>1", b["check"], b["ms_per_step"], b["n_gpus"], b["config"]["parallelism"])
assert a["check"] == b["check"], "summaries differ between N=1 and N>1"
assert a["config"]["edge_entities"] == b["config"]["edge_entities"] and a["config"]["vertices"] == b["config"]["vertices"]
print("checks equal")
PY
