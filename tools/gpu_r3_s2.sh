# fast parity on the current build, then the C4 headline: locality order, id order, and the r2 library
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m "gpu and not fullsize" -x -q ${PYTEST_K:-} -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -40 gpurun_out/pytest_fast.log; exit 1; }
tail -2 gpurun_out/pytest_fast.log
B=raphtory_amd/_build/librgpu.so
cp $B gpurun_out/librgpu_new.so
run() {  # name, extra bench args
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass --no-secondary $2 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail -20 gpurun_out/ab_$1.err; return 1; }
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));print(d['ms_per_step'])")"
}
run loc "" && run idord "--vertex-order id" || exit 1
if [ -f abtest/librgpu_${AB_TAG:-r2}.so ]; then
  cp abtest/librgpu_${AB_TAG:-r2}.so $B
  run ${AB_TAG:-r2} ""; rc=$?
  cp gpurun_out/librgpu_new.so $B
  exit $rc
fi
