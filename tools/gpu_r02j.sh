set -o pipefail
mkdir -p gpurun_out/r02j
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r02j/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/traffic.py --out gpurun_out/r02j/traffic.json --tmp gpurun_out/r02j/traffic > gpurun_out/r02j/traffic.log 2>&1 || exit 2
cp gpurun_out/r02j/traffic.json profiles/traffic.json
timeout -k 10 900 python -u bench.py --steps 10 > gpurun_out/r02j/bench_c2.json 2> gpurun_out/r02j/bench_c2.err || exit 3
echo ALL OK
