set -o pipefail
O=gpurun_out/r02ai
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/stream_sweep.py --config c5 --chunks 524288,1048576 --workers 2,3,4 --stream-reads 8000000 > $O/sweep_c5.log 2>&1 || exit 1
timeout -k 10 500 python3 -u tools/stream_sweep.py --config c2 --chunks 524288,1048576 --workers 2,3,4 --stream-reads 8000000 > $O/sweep_c2.log 2>&1 || exit 2
echo ALL OK
