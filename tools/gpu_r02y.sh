set -o pipefail
O=gpurun_out/r02y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 5 60 python -u tools/aln_case.py --lib gpurun_bisect/libsmemgpu_oldfull.so > $O/oldfull.log 2>&1; echo "oldfull rc=$?" >> $O/rc.txt
SMEM_ALN_HEAVY_MIN=0 timeout -k 5 60 python -u tools/aln_case.py --lib gpurun_bisect/libsmemgpu_oldfull.so > $O/oldfull_h0.log 2>&1; echo "oldfull_h0 rc=$?" >> $O/rc.txt
echo DONE
