set -o pipefail
O=gpurun_out/r02o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/stream_sweep.py --chunks 262144,524288,1048576 --workers 2,3,4 --stream-reads 8000000 > $O/sweep_c2.log 2>&1 || exit 1
echo ALL OK
