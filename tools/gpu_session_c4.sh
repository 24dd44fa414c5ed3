# one GPU call: parity with the non-temporal streams, then the same-process A/B of the C4 query
mkdir -p gpurun_out
RGPU_NT=1 timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_nt.log 2>&1 || { tail -30 gpurun_out/pytest_nt.log; exit 1; }
tail -2 gpurun_out/pytest_nt.log
timeout -k 10 700 python -u tools/c4_ab.py ${AB_ARGS:-base: nt:RGPU_NT=1} > gpurun_out/c4_ab.log 2>&1 || exit $?
for v in ${C2_ENV:-RGPU_NT=0 RGPU_NT=1}; do
  env $v timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-edge-counts --steps 5 --warmup 2 > gpurun_out/c2_$v.log 2>&1 || exit $?
done
