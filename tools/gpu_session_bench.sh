# fast parity (default + dense forced), then the full default bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
RGPU_DENSE=1000 timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1 || { tail -30 gpurun_out/pytest_dense.log; exit 1; }
tail -2 gpurun_out/pytest_dense.log
timeout -k 10 700 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log > gpurun_out/bench_final.json
