# P = 1 vs 8 rehearsal of the partitioned C4 query on the 300M-update prefix (tools/part_sim.py)
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/part_sim.py --interactions 100000000 --parts ${PARTS:-1,8} > gpurun_out/part_sim_300m.jsonl 2> gpurun_out/part_sim_300m.err; rc=$?
tail -5 gpurun_out/part_sim_300m.err
python - <<'PY'
import json
for l in open("gpurun_out/part_sim_300m.jsonl"):
    d = json.loads(l)
    print(d["P"], "kernel max", d["kernel_ms_max"], "total", d["kernel_ms_total"], "k+x max", d["kernel_plus_xchg_ms_max"],
          "xchg MB", d["xchg_MB_per_query"], "by kernel", d["kernel_ms_sum_by_kernel"], "check", d["check"])
PY
exit $rc
