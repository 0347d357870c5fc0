# round-6 scratch driver: dense SA with / without the shared pool (eight handles), then the giant split with priority
mkdir -p gpurun_out/s6p
timeout -k 10 900 python -u tools/flaky_probe.py --reps 20 --settings ctx8_t16_b37_pool_check,ctx8_t16_b37_check --out gpurun_out/s6p/flaky.json > gpurun_out/s6p/flaky.log 2>&1 || exit 1
bash tools/gpu_run.sh s6p "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=128/SMEM_ALN_GIANTS=32/SMEM_ALN_GIANTS=512" && echo "ALL OK s6p"
