# chaining: tests, then per-read cycles and a giant_min / rest-LDS sweep
set -o pipefail
O=gpurun_out/${CHAIN_OUT:-chain5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for P in uniform human; do
  SMEM_CHAIN_DBG=1 timeout -k 10 500 python -u tools/chain_prof.py --genome-profile $P --sweep "${SWEEP:-1024:36}" > $O/chain_$P.json 2> $O/chain_$P.err || exit 2
done
echo ALL OK
