# round 6: hub threshold at P = 8 on the 1B graph (RGPU_HEAVY per process; read at seal) — HS values
set -u
mkdir -p gpurun_out
for h in ${HS:-600 1200}; do
  RGPU_SLOTS=1 RGPU_HEAVY=$h timeout -k 10 ${SECS:-330} python -u tools/part_sim.py --interactions ${INTER:-333333334} --parts 8 --probe-rounds 0 --profile-rounds 1 > gpurun_out/part_heavy${h}_r6.jsonl 2> gpurun_out/part_heavy${h}_r6.err; rc=$?
  echo "heavy=$h rc=$rc"; grep -o '"kernel_ms_max": [0-9.]*' gpurun_out/part_heavy${h}_r6.jsonl; [ $rc -ne 0 ] && exit $rc
done
exit 0
