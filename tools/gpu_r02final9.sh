# c3 / c4 / c5 on the final build (DESIGN table from one build)
set -o pipefail
O=gpurun_out/final9
mkdir -p $O
export TMPDIR=/tmp
for c in c3 c4 c5; do
  timeout -k 10 600 python -u bench.py --steps 10 --config $c --side-stages 0 > $O/bench_$c.json 2> $O/bench_$c.err || exit 2
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 300 --timeout-method thread > $O/chain_tests.log 2>&1 || exit 3
echo ALL OK
