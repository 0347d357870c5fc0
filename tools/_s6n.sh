# round-6 scratch driver: giant split with priority; the eight-context failure by init setting
mkdir -p gpurun_out/s6n
bash tools/gpu_run.sh s6n "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=128/SMEM_ALN_GIANTS=32/SMEM_ALN_GIANTS=512" || exit 1
timeout -k 10 900 python -u tools/flaky_probe.py --reps 8 --settings ctx8_t16_b37,ctx8_t16_b37_syncinit,ctx8_t16_b37_walk,ctx8_t16_b37_saraw,ctx2_t16_b37,ctx8_t16_b37_guard --out gpurun_out/s6n/flaky.json > gpurun_out/s6n/flaky.log 2>&1 && echo "ALL OK s6n"
