# round-6 scratch driver: device buffer overrun guards on the eight-context failure
mkdir -p gpurun_out/s6k
timeout -k 10 600 python -u tools/flaky_probe.py --reps 3 --settings ctx1_t1_b37_guard,ctx1_t16_b37_guard,ctx8_t8_b37_guard --out gpurun_out/s6k/flaky.json > gpurun_out/s6k/flaky.log 2>&1 && echo "ALL OK s6k"
