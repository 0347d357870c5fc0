# round-6 scratch driver: the 256-column lane tier -- alignment parity tests, then c4's stage time
mkdir -p gpurun_out/s6y
bash tools/gpu_run.sh s6y "tests:aln,or,ksw,or,chain2aln" "aln:--launches,2,--config,c4" "aln:--launches,2" && echo "ALL OK s6y"
