# round-6 scratch driver: GPU suite (no -x), then the walk A/B (regions compared across settings) and the replay ceiling
mkdir -p gpurun_out/s6e
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/s6e/tests.log 2>&1
echo "tests rc $?"
tail -n 3 gpurun_out/s6e/tests.log
bash tools/gpu_run.sh s6e "aln:--launches,2,--compare,--env-sweep,SMEM_ALN_WALK_ORDER=0/SMEM_ALN_WALK_WAVES=4/SMEM_ALN_WALK_WAVES=8/SMEM_ALN_WALK_WAVES=12" \
  py:tools/replay_ceiling.py:--reads,200000,--out,gpurun_out/s6e/replay_human.json
