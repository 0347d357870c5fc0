# variant 24 (backward-step bookkeeping as selects) vs the default, same process
set -o pipefail
O=gpurun_out/r02bl
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "variant" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 700 python -u tools/sweep.py --genome-mbp 3101.804739 --lanes 768 --reps 5 --variants 2,24,2,24 > $O/sweep.jsonl 2> $O/sweep.err || exit 2
echo ALL OK
