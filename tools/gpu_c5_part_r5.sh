# round-5 GPU: the C5 live bench and the P = 1 / 8 partitioned rehearsal on the 300M prefix (with the
# RCCL fixed-round probe), on the round-5 kernels
mkdir -p gpurun_out && timeout -k 10 420 python -u bench.py --config c5 > gpurun_out/bench_c5_r5.json 2> gpurun_out/bench_c5_r5.err; rc=$?; tail -c 600 gpurun_out/bench_c5_r5.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/part_sim.py --interactions 100000000 --parts 1,8 --probe-rounds 500 --profile-rounds 1 > gpurun_out/part_sim_p1p8_300m_r5final.jsonl 2> gpurun_out/part_sim_r5final.err; rc=$?; tail -c 1500 gpurun_out/part_sim_p1p8_300m_r5final.jsonl; exit $rc
