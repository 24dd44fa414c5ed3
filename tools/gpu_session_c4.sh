# one GPU call: same-process A/B of the C4 query's launch knobs (tools/c4_ab.py)
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/c4_ab.py ${AB_ARGS:-base: g8k:RGPU_STEP_GRID=8192 c16:RGPU_CHUNK0=16,RGPU_CHUNK=12 d3:RGPU_DENSE=3 d6:RGPU_DENSE=6} > gpurun_out/c4_ab.log 2>&1 || exit $?
