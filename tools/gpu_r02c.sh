set -o pipefail
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02c/stream_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --steps 10 --cpu-seconds 0 --side-stages 0 --stream-reads 4000000 > gpurun_out/r02c/bench_c2_stream4m.json 2> gpurun_out/r02c/bench_c2.err || exit 2
timeout -k 10 900 python -u bench.py --steps 10 --config c5 --cpu-seconds 0 --side-stages 0 > gpurun_out/r02c/bench_c5.json 2> gpurun_out/r02c/bench_c5.err || exit 3
echo ALL OK
