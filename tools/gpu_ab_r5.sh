# round-5 GPU: one same-process A/B of env settings on the 1B graph (tools/ab.py); AB_SETTINGS and AB_TAG name it
# e.g. AB_SETTINGS="base,RGPU_LONG_RATIO=2" AB_TAG=long_ratio bash tools/gpu_ab_r5.sh
set -u
S="${AB_SETTINGS:-base,RGPU_LONG_RATIO=2,RGPU_LONG_RATIO=8}"
T="${AB_TAG:-ab_r5}"
mkdir -p gpurun_out && timeout -k 10 600 python -u tools/ab.py --settings "$S" --rounds 2 --profile > "gpurun_out/$T.jsonl" 2> "gpurun_out/$T.err"; rc=$?; cat "gpurun_out/$T.jsonl"; exit $rc
