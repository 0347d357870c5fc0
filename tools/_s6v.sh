# round-6 scratch driver: c4 / c5 (streaming ratio)
mkdir -p gpurun_out/s6v
bash tools/gpu_run.sh s6v "bench:--config,c4,--e2e-reads,0,--cpu-seconds,0,--other-profile,0" "bench:--config,c5,--e2e-reads,0,--cpu-seconds,0,--other-profile,0" && echo "ALL OK s6v"
