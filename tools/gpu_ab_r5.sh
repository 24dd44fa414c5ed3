# round-5 GPU: the dense-superstep divisor on the round-5 kernels (RGPU_DENSE; default 4)
mkdir -p gpurun_out && timeout -k 10 600 python -u tools/ab.py --settings "base,RGPU_DENSE=2,RGPU_DENSE=8,RGPU_DENSE=16" --rounds 2 --profile > gpurun_out/ab_dense_r5.jsonl 2> gpurun_out/ab_dense_r5.err; rc=$?; cat gpurun_out/ab_dense_r5.jsonl; exit $rc
