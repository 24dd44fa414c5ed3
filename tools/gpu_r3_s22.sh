# fast GPU suite, then the default bench line (as the driver runs it)
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -40 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
timeout -k 10 660 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
tail -c 4000 gpurun_out/bench_default.json
