# one GPU call: fast parity tests, then the same-process A/B of the C4 query (tools/c4_ab.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
timeout -k 10 420 python -u tools/c4_ab.py ${AB_VARIANTS:-base: nocb:RGPU_CHGBITS=0} > gpurun_out/c4_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/c2.log 2>&1 || exit $?
