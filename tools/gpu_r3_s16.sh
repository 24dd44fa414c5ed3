# partitioned GPU tests, then the P = 1 vs 8 rehearsal with the exchange kernels timed
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dense.py tests/test_gpu_live.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_part.log 2>&1 || { tail -30 gpurun_out/pytest_part.log; exit 1; }
tail -2 gpurun_out/pytest_part.log
PARTS=${PARTS:-1,8} bash tools/gpu_r3_part.sh
python -c "
import json
for l in open('gpurun_out/part_sim_300m.jsonl'):
    d=json.loads(l); print(d['P'], d['kernel_ms_per_partition'], d.get('serial_wall_ms_per_partition')); print(d['partition0_kernels'])"
