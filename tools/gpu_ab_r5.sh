# round-5 GPU: same-box A/B of non-temporal slot-stream loads in the long superstep form
mkdir -p gpurun_out && RGPU_STEP_OPTS=15 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider tests/test_gpu_step_forms.py > gpurun_out/pytest_nt.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_nt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/ab.py --settings "base,RGPU_STEP_OPTS=15" --rounds 2 --profile > gpurun_out/ab_nt_c4.jsonl 2> gpurun_out/ab_nt_c4.err; rc=$?; cat gpurun_out/ab_nt_c4.jsonl; exit $rc
