# round-6 scratch driver: giant split with the third stream at the highest priority
mkdir -p gpurun_out/s6m
bash tools/gpu_run.sh s6m "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=128/SMEM_ALN_GIANTS=32/SMEM_ALN_GIANTS=512/SMEM_ALN_GIANTS=1024" && echo "ALL OK s6m"
