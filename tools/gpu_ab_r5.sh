# round-5 GPU check: parity suites, a same-box A/B of the hub prologue width, and the per-step
# C4 work trace (non-lean: visited / slots / gathers per superstep)
mkdir -p gpurun_out && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_batch_modes.py tests/test_gpu_heavy.py tests/test_gpu_parity.py tests/test_gpu_partitioned.py tests/test_gpu_vertex_program.py tests/test_gpu_configs.py::test_c5_live_at_size_vs_oracle > gpurun_out/pytest_r5e.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5e.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/ab.py --settings "base,RGPU_HUB_PRO=16" --rounds 2 --profile > gpurun_out/ab_r5e.jsonl 2> gpurun_out/ab_r5e.err; rc=$?; cat gpurun_out/ab_r5e.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/c4_trace.py --out gpurun_out/c4_trace_full.csv > gpurun_out/c4_trace_full.txt 2>&1; rc=$?; tail -22 gpurun_out/c4_trace_full.txt | cut -c1-330; exit $rc
