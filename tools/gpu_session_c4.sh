# one GPU call: fast parity tests (default, and with visit-all steps forced + uniform-words-first +
# grouped K2 prefetch), then the same-process A/B of the C4 query (tools/c4_ab.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
RGPU_DENSE=1000 RGPU_UWFIRST=1 RGPU_SLOTS_GROUP=4 timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1 || { tail -30 gpurun_out/pytest_dense.log; exit 1; }
tail -2 gpurun_out/pytest_dense.log
RGPU_SLOTS_GROUP=2 timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_g2.log 2>&1 || { tail -30 gpurun_out/pytest_g2.log; exit 1; }
tail -2 gpurun_out/pytest_g2.log
timeout -k 10 700 python -u tools/c4_ab.py ${AB_ARGS:-base: uwf:RGPU_UWFIRST=1 g2:RGPU_SLOTS_GROUP=2 g4:RGPU_SLOTS_GROUP=4} > gpurun_out/c4_ab.log 2>&1 || exit $?
