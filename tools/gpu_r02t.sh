set -o pipefail
O=gpurun_out/r02t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/aln_prof.py --launches 2 > $O/warm.log 2>&1 || exit 1
PMC_PROG=tools/aln_prof.py PMC_KERNEL=aln_kernel PMC_PASSES="1 2" timeout -k 10 600 bash tools/pmc_passes.sh $O/pmc --launches 1 > $O/pmc.log 2>&1 || exit 2
echo ALL OK
