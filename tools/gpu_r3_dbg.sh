mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_partitioned.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_dbg.log
if [ $rc -eq 1 ]; then
  RGPU_TSG=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_partitioned.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_dbg2.log 2>&1; echo "TSG=0 rc=$?"; tail -3 gpurun_out/pytest_dbg2.log
fi
