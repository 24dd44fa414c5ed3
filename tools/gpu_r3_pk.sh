# rocprofv3 kernel trace of the P = 8 loopback rehearsal (every kernel, the exchange kernels too)
mkdir -p gpurun_out/pk
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pk -o run --output-format csv -- python3 tools/part_sim.py --interactions ${INTER:-33333334} --parts ${PARTS:-8} > gpurun_out/pk/run.log 2>&1; rc=$?
tail -3 gpurun_out/pk/run.log
python3 - <<'PY'
import csv, glob
fs = glob.glob("gpurun_out/pk/**/*kernel_stats.csv", recursive=True)
for f in fs:
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:25]:
        print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):7d} {r["Name"][:110]}')
PY
exit $rc
