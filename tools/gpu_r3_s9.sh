# fast GPU suite, same-process C4 A/B (inline edge bits, dense K2), then the P = 1 vs 8 rehearsal
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m "gpu and not fullsize" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -40 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log

timeout -k 10 700 python -u tools/c4_ab.py --steps 2 ${AB:-base: notsg:RGPU_TSG=0} > gpurun_out/c4_ab.log 2>&1 || { tail -20 gpurun_out/c4_ab.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/c4_ab.log"):
    l = l.strip()
    if not l.startswith("{"):
        print(l); continue
    d = json.loads(l); k = d["kernels"]
    print(d["variant"], d["round"], d["ms"], d["same"], {n: k[n] for n in k})
PY
[ -n "${NOPART:-}" ] || PARTS=1,8 bash tools/gpu_r3_part.sh
