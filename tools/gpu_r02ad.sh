set -o pipefail
O=gpurun_out/r02ad
mkdir -p $O
export TMPDIR=/tmp
for hs in 1000000 128 48; do
  SMEM_ALN_HEAVY_SEEDS=$hs timeout -k 10 300 python -u tools/aln_prof.py --launches 2 > $O/u_$hs.log 2>&1 || exit 1
  SMEM_ALN_HEAVY_SEEDS=$hs timeout -k 10 300 python -u tools/aln_prof.py --launches 2 --genome-profile human > $O/h_$hs.log 2>&1 || exit 2
done
SMEM_ALN_HEAVY_MIN=9 SMEM_ALN_HEAVY_SEEDS=1000000 timeout -k 10 300 python -u tools/aln_prof.py --launches 2 --genome-profile human > $O/h_m9.log 2>&1 || exit 3
SMEM_ALN_HEAVY_MIN=33 SMEM_ALN_HEAVY_SEEDS=1000000 timeout -k 10 300 python -u tools/aln_prof.py --launches 2 --genome-profile human > $O/h_m33.log 2>&1 || exit 4
echo ALL OK
