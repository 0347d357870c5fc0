set -o pipefail
O=gpurun_out/r02p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t1m -o s -- python3 -u tools/stream_sweep.py --chunks 1048576 --workers 2 --stream-reads 8000000 > $O/t1m.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t512k -o s -- python3 -u tools/stream_sweep.py --chunks 524288 --workers 4 --stream-reads 8000000 > $O/t512k.log 2>&1 || exit 2
echo ALL OK
