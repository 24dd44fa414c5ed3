# live-ingest tests (device delta packer) first, then the C4 profile pass in both vertex orders
# (+ a reference library), then the fast GPU suite
mkdir -p gpurun_out
B=raphtory_amd/_build/librgpu.so
cp $B gpurun_out/librgpu_new.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_live.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_live.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_live.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
prof() {  # name, lib, bench args
  cp $2 $B
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-edge-counts $3 > gpurun_out/prof_$1.json 2> gpurun_out/prof_$1.err || { tail -20 gpurun_out/prof_$1.err; cp gpurun_out/librgpu_new.so $B; return 1; }
  python - "$1" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/prof_{v}.json"))
print(v, d["ms_per_step"], {k: (x.get("launches"), x.get("ms"), x.get("GBps")) for k, x in d.get("kernels", {}).items()})
PY
}
prof loc gpurun_out/librgpu_new.so "" && prof id gpurun_out/librgpu_new.so "--vertex-order id" && { [ -z "${AB_TAG:-}" ] || prof $AB_TAG abtest/librgpu_$AB_TAG.so ""; }
rc=$?
cp gpurun_out/librgpu_new.so $B
[ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python -u -m pytest tests -m "gpu and not fullsize" -q -p no:cacheprovider --maxfail 10 --deselect tests/test_gpu_live.py --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -60 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
