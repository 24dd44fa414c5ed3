# fast GPU suite, then the P = 1 vs 8 rehearsal
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -40 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
PARTS=1,8 bash tools/gpu_r3_part.sh
python -c "
import json
for l in open('gpurun_out/part_sim_300m.jsonl'):
    d=json.loads(l); print(d['P'], d['kernel_ms_per_partition']); print(d['partition0_kernels']); print(d.get('kernel_GB_sum_by_kernel'))"
