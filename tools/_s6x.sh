# round-6 scratch driver: e2e (bwa-gpu mem, 62.5k-read worker batches) with / without the giant split
mkdir -p gpurun_out/s6x
Q="bench:--side-stages,0,--cpu-seconds,0,--other-profile,0,--parity,0,--e2e-pairs,0,--e2e-chunk-reads,0"
bash tools/gpu_run.sh s6x "$Q" || exit 1
SMEM_ALN_GIANTS=0 bash tools/gpu_run.sh s6x_g0 "$Q" || exit 1
bash tools/gpu_run.sh s6x2 "$Q" && echo "ALL OK s6x"
