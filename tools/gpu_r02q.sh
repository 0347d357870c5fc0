set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/stream_sweep.py --chunks 131072,262144,524288,1048576 --workers 2,3,4 --stream-reads 8000000 > $O/sweep_c2.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t512k -o s -- python3 -u tools/stream_sweep.py --chunks 524288 --workers 4 --stream-reads 8000000 > $O/t512k.log 2>&1 || exit 3
echo ALL OK
