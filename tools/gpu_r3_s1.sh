# fast parity on the current build, then the same-box A/B of the headline against abtest/librgpu_$AB_TAG.so
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -30 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
ROUNDS=${ROUNDS:-1} bash tools/ab_lib.sh
