# round-6 scratch driver: the headline step after the lazy third stream (quick legs)
mkdir -p gpurun_out/s6t
bash tools/gpu_run.sh s6t "bench:--side-stages,0,--cpu-seconds,0,--e2e-reads,0,--other-profile,0,--parity,0" "aln:--launches,2" && echo "ALL OK s6t"
