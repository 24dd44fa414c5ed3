# the whole GPU suite (full-size configs included), as the driver runs it
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_full.log
exit $rc
