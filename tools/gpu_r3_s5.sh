# live ingest (device + partitioned merges), analysis tasks, then the C4 profile pass in both orders
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_live.py tests/test_gpu_analysis_tasks.py -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_live.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_live.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
prof() {  # name, bench args
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-edge-counts $2 > gpurun_out/prof_$1.json 2> gpurun_out/prof_$1.err || { tail -20 gpurun_out/prof_$1.err; return 1; }
  python - "$1" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/prof_{v}.json"))
print(v, d["ms_per_step"], {k: (x.get("launches"), x.get("ms"), x.get("GBps")) for k, x in d.get("kernels", {}).items()})
PY
}
prof loc "" && prof id "--vertex-order id"
