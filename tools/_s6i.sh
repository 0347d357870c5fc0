# round-6 scratch driver: giant split after the prep-atomic fix; the eight-context integration test x4 (host crash trace on)
bash tools/gpu_run.sh s6i "aln:--launches,3,--compare,--env-sweep,SMEM_ALN_GIANTS=0/SMEM_ALN_GIANTS=128/SMEM_ALN_GIANTS=32/SMEM_ALN_GIANTS=512" || exit 1
for k in 1 2 3 4; do
  timeout -k 10 600 python -u -m pytest tests/test_bwa_integration.py -m gpu -x -q --timeout 300 --timeout-method thread -k eight_contexts > gpurun_out/s6i/eight_$k.log 2>&1 || { echo "eight contexts failed at $k"; exit 2; }
done
bash tools/gpu_run.sh s6i tests && echo "ALL OK s6i"
