# round-6 scratch driver: the driver's bench line (defaults) and the seeding kernel's rocprof summary
mkdir -p gpurun_out/s6s
bash tools/gpu_run.sh s6s bench rocprof && echo "ALL OK s6s"
