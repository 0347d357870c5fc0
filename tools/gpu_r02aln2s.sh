# chains -> regions with the light reads' kernel beside the heavy reads'
# kernels (SMEM_ALN_STREAMS=2, default) vs one after the other (1), and the
# light waves' claims before they exit (SMEM_ALN_LIGHT_CLAIMS)
set -o pipefail
O=gpurun_out/aln2s_b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_aln.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
SW="SMEM_ALN_STREAMS=1;SMEM_ALN_STREAMS=2,SMEM_ALN_LIGHT_CLAIMS=0;SMEM_ALN_STREAMS=2,SMEM_ALN_LIGHT_CLAIMS=1;SMEM_ALN_STREAMS=2,SMEM_ALN_LIGHT_CLAIMS=2;SMEM_ALN_STREAMS=2,SMEM_ALN_LIGHT_CLAIMS=4;SMEM_ALN_STREAMS=2,SMEM_ALN_LIGHT_CLAIMS=16;SMEM_ALN_STREAMS=1"
for P in uniform human; do
  echo "== $P" >> $O/aln.log
  timeout -k 10 500 python -u tools/aln_prof.py --launches 3 --env-sweep "$SW" --genome-profile $P >> $O/aln.log 2>&1 || exit 2
done
echo ALL OK
