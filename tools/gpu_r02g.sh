set -o pipefail
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r02g/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --steps 10 > gpurun_out/r02g/bench_c2.json 2> gpurun_out/r02g/bench_c2.err || exit 2
echo ALL OK
