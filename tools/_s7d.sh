# round-6 scratch driver: the light reads' passes forked before the heavy chains' short SW -- parity, c4 / c2 stage times
mkdir -p gpurun_out/s7d
bash tools/gpu_run.sh s7d "tests:aln,or,ksw,or,chain2aln,or,bwa_integration" "aln:--launches,2,--config,c4" "aln:--launches,3" && echo "ALL OK s7d"
