set -o pipefail
O=gpurun_out/r02ap
mkdir -p $O
export TMPDIR=/tmp
SMEM_ALN_SPEC_LOCAL=1 timeout -k 10 300 python -u -m pytest tests/test_aln.py -m gpu -x -q --timeout 60 --timeout-method thread > $O/gpu_tests_local.log 2>&1 || exit 1
for sl in 0 1; do
SMEM_ALN_SPEC_LOCAL=$sl timeout -k 10 300 python -u tools/aln_prof.py --launches 2 > $O/u_$sl.log 2>&1 || exit 2
SMEM_ALN_SPEC_LOCAL=$sl timeout -k 10 300 python -u tools/aln_prof.py --launches 2 --genome-profile human > $O/h_$sl.log 2>&1 || exit 3
done
echo ALL OK
