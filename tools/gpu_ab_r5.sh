# round-5 GPU: the superstep-form parity test
mkdir -p gpurun_out && timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_step_forms.py > gpurun_out/pytest_step_forms.log 2>&1; rc=$?; tail -12 gpurun_out/pytest_step_forms.log; exit $rc
