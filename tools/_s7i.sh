# round-6 scratch driver: the driver's N > 1 launch line rehearsed (two ranks sharing the one GPU)
mkdir -p gpurun_out/s7i
bash tools/gpu_run.sh s7i "dist2:--steps,5,--warmup,2" && echo "ALL OK s7i"
