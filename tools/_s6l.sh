# round-6 scratch driver: giant split (now active in Python batches) + the eight-context failure under host ASan
mkdir -p gpurun_out/s6l
bash tools/gpu_run.sh s6l "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=128/SMEM_ALN_GIANTS=32/SMEM_ALN_GIANTS=512" || exit 1
timeout -k 10 900 python -u tools/flaky_probe.py --bwa oracle/_ref/bwa-gpu-asan --reps 8 --settings ctx8_t16_b37,ctx8_t8_b37 --out gpurun_out/s6l/flaky.json > gpurun_out/s6l/flaky.log 2>&1 && echo "ALL OK s6l"
