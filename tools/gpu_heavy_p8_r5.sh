# round-5 GPU: hub threshold at P = 8 (300M prefix) on the round-5 kernels: slowest partition per RGPU_HEAVY
mkdir -p gpurun_out
for h in 256 512 1024 2048; do
  RGPU_HEAVY=$h timeout -k 10 300 python -u tools/part_sim.py --interactions 100000000 --parts 8 --probe-rounds 0 --profile-rounds 1 > gpurun_out/part_sim_heavy${h}_r5.jsonl 2> gpurun_out/part_sim_heavy${h}_r5.err; rc=$?
  echo "heavy=$h rc=$rc"; grep -o '"kernel_ms_max": [0-9.]*' gpurun_out/part_sim_heavy${h}_r5.jsonl; [ $rc -ne 0 ] && exit $rc
done
exit 0
