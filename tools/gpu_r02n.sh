set -o pipefail
O=gpurun_out/r02n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/stream_sweep.py --chunks 131072 --workers 4 --stream-reads 4000000 > $O/sweep_noprof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o s -- python3 -u tools/stream_sweep.py --chunks 131072 --workers 4 --stream-reads 4000000 > $O/sweep.log 2>&1 || exit 2
echo ALL OK
