#!/bin/bash
# Same-box A/B of the headline query: the in-tree librgpu.so against abtest/librgpu_<tag>.so
# (both loaded by the same bench.py), interleaved, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=raphtory_amd/_build/librgpu.so
cp "$B" gpurun_out/librgpu_new.so
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in new ${AB_TAG:-r1}; do
    if [ "$v" = new ]; then cp gpurun_out/librgpu_new.so "$B"; else cp "abtest/librgpu_$v.so" "$B"; fi
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass ${BENCH_ARGS:-} \
      > "gpurun_out/ab_${v}_$i.json" 2> "gpurun_out/ab_${v}_$i.err" || { cp gpurun_out/librgpu_new.so "$B"; exit 1; }
    echo "$v $i $(python -c "import json;print(json.load(open('gpurun_out/ab_${v}_$i.json'))['ms_per_step'])")"
  done
done
cp gpurun_out/librgpu_new.so "$B"
