# session 7 baseline: C4 headline (with its profile pass), then the P = 1 vs 8 rehearsal on the 300M prefix
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/bench_s7.json 2> gpurun_out/bench_s7.err || { tail -30 gpurun_out/bench_s7.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_s7.json"))
print(d["ms_per_step"], {k: (x.get("launches"), x.get("ms"), x.get("GBps")) for k, x in d.get("kernels", {}).items()})
PY
PARTS=1,8 bash tools/gpu_r3_part.sh
