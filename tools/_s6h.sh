# round-6 scratch driver: the giant split (regions identical with it off; the stage's time), then the GPU suite
bash tools/gpu_run.sh s6h "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=128/SMEM_ALN_GIANTS=32/SMEM_ALN_GIANTS=512" tests && echo "ALL OK s6h"
