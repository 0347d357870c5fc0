set -o pipefail
O=gpurun_out/r02s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 10 > $O/bench_c2.json 2> $O/bench_c2.err || exit 2
echo ALL OK
