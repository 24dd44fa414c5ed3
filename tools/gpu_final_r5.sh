# round-5 end: the full GPU suite and smoke() on the final tree
mkdir -p gpurun_out && timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_full_r5end.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_full_r5end.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5end.log 2>&1; rc=$?; tail -3 gpurun_out/smoke_r5end.log; exit $rc
