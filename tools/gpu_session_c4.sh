# one GPU call: fast parity tests (default and with the dense-step rule forced on almost every
# step), then the same-process A/B of the C4 query (tools/c4_ab.py) and a C2 bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
RGPU_DENSE=1000 timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1 || { tail -30 gpurun_out/pytest_dense.log; exit 1; }
tail -2 gpurun_out/pytest_dense.log
timeout -k 10 700 python -u tools/c4_ab.py ${AB_ARGS:-base: w6:RGPU_STEP_VARIANT=68} > gpurun_out/c4_ab.log 2>&1 || exit $?
for v in ${C2_ENV:-RGPU_STEP_VARIANT=4 RGPU_STEP_VARIANT=68}; do
  env $v timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-edge-counts --steps 5 --warmup 2 > gpurun_out/c2_$v.log 2>&1 || exit $?
done
