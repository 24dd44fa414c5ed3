# C4 with 3 (default) and 4 batch slots in flight (RGPU_SLOTS is read at rgpu_open: one process each)
mkdir -p gpurun_out
for v in 3 2 4; do
  RGPU_SLOTS=$v timeout -k 10 330 python -u bench.py --no-cpu-baseline --no-secondary --no-profile-pass --no-edge-counts --steps 5 > gpurun_out/c4_slots$v.log 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4_slots$v.log
done
