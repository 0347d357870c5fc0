set -o pipefail
O=gpurun_out/r02aj
mkdir -p $O
export TMPDIR=/tmp
for sl in 2 99; do
SMEM_STREAM_GPU_SLOTS=$sl timeout -k 10 400 python3 -u tools/stream_sweep.py --config c2 --chunks 524288,1048576 --workers 2,3,4 --stream-reads 8000000 > $O/sweep_c2_s$sl.log 2>&1 || exit 1
done
SMEM_STREAM_GPU_SLOTS=2 timeout -k 10 400 python3 -u tools/stream_sweep.py --config c5 --chunks 524288,1048576 --workers 2,3,4 --stream-reads 8000000 > $O/sweep_c5_s2.log 2>&1 || exit 2
echo ALL OK
