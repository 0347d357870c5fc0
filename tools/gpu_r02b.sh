set -o pipefail
mkdir -p gpurun_out/r02b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b/stream_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --steps 10 > gpurun_out/r02b/bench_c2.json 2> gpurun_out/r02b/bench_c2.err || exit 2
timeout -k 10 600 python -u tools/traffic.py --out gpurun_out/r02b/traffic.json --tmp gpurun_out/r02b/traffic > gpurun_out/r02b/traffic.log 2>&1 || exit 3
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r02b/prof -o bench -- python -u bench.py --steps 10 --cpu-seconds 0 > gpurun_out/r02b/bench_c2_under_rocprof.json 2> gpurun_out/r02b/bench_c2_rocprof.err || exit 4
echo ALL OK
