# round-6 scratch driver: GPU suite, uniform-profile alignment with / without the giant split, eight-handle probe
mkdir -p gpurun_out/s6r
bash tools/gpu_run.sh s6r tests "aln:--launches,3,--compare,--genome-profile,uniform,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=2048" || exit 1
timeout -k 10 600 python -u tools/flaky_probe.py --reps 10 --settings ctx8_t16_b37,ctx8_t8_b37 --out gpurun_out/s6r/flaky.json > gpurun_out/s6r/flaky.log 2>&1 && echo "ALL OK s6r"
