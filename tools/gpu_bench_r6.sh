# round 6: the default bench line (the driver's command) -> gpurun_out/bench_$TAG.json (+ .err progress)
T="${TAG:-r6}"
mkdir -p gpurun_out && timeout -k 10 ${SECS:-1000} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err; rc=$?
tail -c 600 gpurun_out/bench_$T.json; tail -3 gpurun_out/bench_$T.err; exit $rc
