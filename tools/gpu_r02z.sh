set -o pipefail
O=gpurun_out/r02za
mkdir -p $O
export TMPDIR=/tmp
timeout -k 5 40 python -u tools/aln_case.py --lib gpurun_bisect/libsmemgpu_F.so > $O/F.log 2>&1; echo "F rc=$?" >> $O/rc.txt
SMEM_ALN_HEAVY_MIN=1 timeout -k 5 40 python -u tools/aln_case.py --lib gpurun_bisect/libsmemgpu_F.so > $O/F_h1.log 2>&1; echo "F_h1 rc=$?" >> $O/rc.txt
for fx in g1_k14s20_tight g2_default_std g2_k14s20_std; do SMEM_ALN_HEAVY_MIN=1 timeout -k 5 40 python -u tools/aln_case.py --fix $fx --lib gpurun_bisect/libsmemgpu_F.so > $O/F_h1_$fx.log 2>&1; echo "F_h1_$fx rc=$?" >> $O/rc.txt; done
echo DONE
