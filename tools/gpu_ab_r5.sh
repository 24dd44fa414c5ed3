# round-5 GPU: a quick parity check of the final library
mkdir -p gpurun_out && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_step_forms.py tests/test_gpu_parity.py tests/test_gpu_heavy.py tests/test_gpu_batch_modes.py > gpurun_out/pytest_final_quick.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_final_quick.log; exit $rc
