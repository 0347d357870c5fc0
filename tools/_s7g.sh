# round-6 scratch driver: e2e with the fast exit (and without), integration tests
mkdir -p gpurun_out/s7g
Q="bench:--side-stages,0,--cpu-seconds,0,--other-profile,0,--parity,0"
bash tools/gpu_run.sh s7g "tests:bwa_integration" "$Q" || exit 1
SMEM_GPU_FAST_EXIT=0 bash tools/gpu_run.sh s7g_f0 "$Q" && echo "ALL OK s7g"
