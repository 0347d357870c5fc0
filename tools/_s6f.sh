# round-6 scratch driver: request-ceiling sweep, bench, alignment kernel trace
mkdir -p gpurun_out/s6f
timeout -k 10 300 bash tools/ceiling_sweep.sh > gpurun_out/s6f/ceiling_sweep.jsonl 2> gpurun_out/s6f/ceiling_sweep.err || { echo "sweep failed"; exit 1; }
echo "sweep ok"
export SMEM_GPU_MEMORY_DETAIL=1
bash tools/gpu_run.sh s6f bench "aln:--launches,2"
timeout -k 10 600 python -u tools/stream_sweep.py --config c5 --chunks 1048576,2097152 --workers 3,4,6 > gpurun_out/s6f/stream_c5.jsonl 2> gpurun_out/s6f/stream_c5.err || { echo "stream sweep failed"; exit 1; }
SMEM_STREAM_GPU_SLOTS=3 timeout -k 10 600 python -u tools/stream_sweep.py --config c5 --chunks 1048576 --workers 4,6 > gpurun_out/s6f/stream_c5_slots3.jsonl 2> gpurun_out/s6f/stream_c5_slots3.err || { echo "stream sweep 2 failed"; exit 1; }
echo "ALL OK s6f"
