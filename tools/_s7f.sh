# round-6 scratch driver: e2e with / without the HIP runtime prewarm thread
mkdir -p gpurun_out/s7f
Q="bench:--side-stages,0,--cpu-seconds,0,--other-profile,0,--parity,0,--e2e-pairs,0,--e2e-chunk-reads,0"
bash tools/gpu_run.sh s7f "$Q" || exit 1
SMEM_GPU_PREWARM=0 bash tools/gpu_run.sh s7f_p0 "$Q" || exit 1
bash tools/gpu_run.sh s7f2 "$Q" && echo "ALL OK s7f"
