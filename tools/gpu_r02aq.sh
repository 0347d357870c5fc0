set -o pipefail
O=gpurun_out/r02aq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --genome-mbp 3101.804739 --lanes 768 --reps 5 --variants 2,2 > $O/sweep.jsonl 2> $O/sweep.err || exit 2
echo ALL OK
