# partitioned live test, then same-process A/B of the K2 / superstep dealing on one sealed C4 graph
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_live.py -v -p no:cacheprovider -k partitioned --timeout 150 --timeout-method thread > gpurun_out/pytest_live_part.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_live_part.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 700 python -u tools/c4_ab.py --steps 2 "s64t1:RGPU_DEAL_SLOTS=64,RGPU_DEAL_STEP=1" "s16t1:RGPU_DEAL_SLOTS=16,RGPU_DEAL_STEP=1" "s1t1:RGPU_DEAL_SLOTS=1,RGPU_DEAL_STEP=1" "s64t4:RGPU_DEAL_SLOTS=64,RGPU_DEAL_STEP=4" "s64t64:RGPU_DEAL_SLOTS=64,RGPU_DEAL_STEP=64" > gpurun_out/c4_ab_deal.log 2>&1; rc=$?
cat gpurun_out/c4_ab_deal.log | python -c "
import json,sys
for l in sys.stdin:
    l=l.strip()
    if not l.startswith('{'): print(l); continue
    d=json.loads(l); k=d['kernels']
    print(d['variant'], d['round'], d['ms'], d['same'], {n: k[n][1] for n in ('cc_slots','cc_step','heavy') if n in k})
"
exit $rc
