# C5 live-ingest line (device delta packer + merge, CC + PR per tick) on one GPU
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err; rc=$?
tail -5 gpurun_out/c5.err
tail -c 2500 gpurun_out/c5.json
exit $rc
