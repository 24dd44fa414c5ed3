# round 6: the secondary lines — C2 rocprofv3 passes (tools/gpu_prof_r6.sh CFG=c2), C3 and C5 bench lines
set -u
mkdir -p gpurun_out
CFG=c2 STEP_SECS=240 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_prof_r6.sh || exit $?
timeout -k 10 400 python -u bench.py --config c3 --steps 3 > gpurun_out/c3_bench_r6.json 2> gpurun_out/c3_bench_r6.err || exit $?
tail -c 400 gpurun_out/c3_bench_r6.json
timeout -k 10 500 python -u bench.py --config c5 > gpurun_out/c5_bench_r6.json 2> gpurun_out/c5_bench_r6.err || exit $?
tail -c 600 gpurun_out/c5_bench_r6.json
