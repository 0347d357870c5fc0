# round-6 scratch driver: the final tree -- GPU suite, smoke, the driver's bench line, rocprof of the seeding steps
mkdir -p gpurun_out/s6z
bash tools/gpu_run.sh s6z tests smoke bench rocprof && echo "ALL OK s6z"
