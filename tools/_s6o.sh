# round-6 scratch driver: the eight-context failure -- dense SA checked with the shared pool (old) and without (new)
mkdir -p gpurun_out/s6o
timeout -k 10 900 python -u tools/flaky_probe.py --reps 20 --settings ctx8_t16_b37_pool_check,ctx8_t16_b37_check --out gpurun_out/s6o/flaky.json > gpurun_out/s6o/flaky.log 2>&1 && echo "ALL OK s6o"
