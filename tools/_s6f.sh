# round-6 scratch driver: request-ceiling sweep, bench, alignment kernel trace
mkdir -p gpurun_out/s6f
timeout -k 10 300 bash tools/ceiling_sweep.sh > gpurun_out/s6f/ceiling_sweep.jsonl 2> gpurun_out/s6f/ceiling_sweep.err || { echo "sweep failed"; exit 1; }
echo "sweep ok"
export SMEM_GPU_MEMORY_DETAIL=1
bash tools/gpu_run.sh s6f bench "aln:--launches,2"
