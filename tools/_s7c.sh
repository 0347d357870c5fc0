# round-6 scratch driver: the eight-context tests (dense-SA digests), then c4 / c5 with 256k-chunk streaming
mkdir -p gpurun_out/s7c
bash tools/gpu_run.sh s7c "tests:eight_contexts" "bench:--config,c4,--e2e-reads,0,--cpu-seconds,0,--other-profile,0" "bench:--config,c5,--e2e-reads,0,--cpu-seconds,0,--other-profile,0" && echo "ALL OK s7c"
