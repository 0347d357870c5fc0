# round-6 scratch driver: integration tests, then the driver's default bench line
mkdir -p gpurun_out/s6w
bash tools/gpu_run.sh s6w "tests:bwa_integration,or,faults,or,configs" bench && echo "ALL OK s6w"
