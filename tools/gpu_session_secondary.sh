# the dense-step tests, then secondary evidence: the P = 1..8 loopback rehearsal, then the C3 and C5 bench lines
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_dense_file.log 2>&1 || { tail -30 gpurun_out/pytest_dense_file.log; exit 1; }
tail -3 gpurun_out/pytest_dense_file.log
timeout -k 10 500 python -u tools/part_sim.py --parts 1,2,4,8 > gpurun_out/part_sim_final.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --config c3 --steps 2 > gpurun_out/c3_final.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --config c5 > gpurun_out/c5_final.log 2>&1 || exit $?
