# round-6 scratch driver: full GPU suite without -x (a flaky SAM case must not hide the rest), then the measurement steps
mkdir -p gpurun_out/s6d
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/s6d/tests.log 2>&1
echo "tests rc $?"
tail -n 3 gpurun_out/s6d/tests.log
export SMEM_GPU_MEMORY_DETAIL=1
bash tools/gpu_run.sh s6d traffic traffic:--genome-profile,uniform bench env:SMEM_ALN_STATS=1 aln:--launches,3
