set -o pipefail
O=gpurun_out/r02an
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_aln.py -m gpu -x -q --timeout 60 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/aln_prof.py --launches 2 > $O/u.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/aln_prof.py --launches 2 --genome-profile human > $O/h.log 2>&1 || exit 3
echo ALL OK
