# round-6 scratch driver: the final tree again -- GPU suite, smoke, the driver's bench line, rocprof
mkdir -p gpurun_out/s7e
bash tools/gpu_run.sh s7e tests smoke bench rocprof && echo "ALL OK s7e"
