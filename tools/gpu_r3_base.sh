# round-3 baseline on a fresh box: fast parity + recovery test, then the default bench line
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_base.log 2>&1 || { tail -30 gpurun_out/bench_base.log; exit 1; }
tail -c 3000 gpurun_out/bench_base.log
