# round 6: the full GPU suite and smoke() on the current tree (TAG names the logs)
T="${TAG:-r6}"
mkdir -p gpurun_out && timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$T.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1; rc=$?; tail -3 gpurun_out/smoke_$T.log; exit $rc
