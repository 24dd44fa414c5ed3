# round-5 GPU: same-box A/B of the changed-bit probe (RGPU_CBF) on the round-5 superstep kernel
mkdir -p gpurun_out && timeout -k 10 500 python -u tools/ab.py --settings "base,RGPU_CBF=1" --rounds 2 --profile > gpurun_out/ab_cbf2_c4.jsonl 2> gpurun_out/ab_cbf2_c4.err; rc=$?; cat gpurun_out/ab_cbf2_c4.jsonl; exit $rc
