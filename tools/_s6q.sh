# round-6 scratch driver: giants first (passes + candidate index before the other lists' passes)
mkdir -p gpurun_out/s6q
bash tools/gpu_run.sh s6q "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=1024+SMEM_ALN_GIANT_FIRST=2/SMEM_ALN_GIANTS=2048+SMEM_ALN_GIANT_FIRST=2/SMEM_ALN_GIANTS=4096+SMEM_ALN_GIANT_FIRST=2/SMEM_ALN_GIANTS=40000+SMEM_ALN_GIANT_FIRST=2/SMEM_ALN_GIANTS=2048+SMEM_ALN_GIANT_FIRST=1" && echo "ALL OK s6q"
