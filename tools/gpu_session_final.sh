# fast parity (partitioned included), the P=8 loopback rehearsal, then the rocprofv3 kernel-stats
# and PMC passes of the headline (bench.py --profile-only --no-edge-counts)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
timeout -k 10 300 python -u tools/part_sim.py --parts 8 > gpurun_out/part_sim8.log 2>&1 || exit $?
SKIP_BENCH=1 BENCH_ARGS="--no-edge-counts" bash tools/gpu_profile.sh
