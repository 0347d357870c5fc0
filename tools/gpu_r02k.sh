set -o pipefail
mkdir -p gpurun_out/r02k
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "kmer or variants" --timeout 300 --timeout-method thread > gpurun_out/r02k/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/sweep.py --genome-mbp 3101.804739 --lanes 768 --reps 4 --variants 2,23:8,23:10,23:11,23:12,23:13,23:14 > gpurun_out/r02k/sweep.jsonl 2> gpurun_out/r02k/sweep.err || exit 2
timeout -k 10 600 python -u tools/traffic.py --out gpurun_out/r02k/traffic_kt12.json --tmp gpurun_out/r02k/traffic_kt12 --variant 23 --kmer-k 12 > gpurun_out/r02k/traffic_kt12.log 2>&1 || exit 3
echo ALL OK
