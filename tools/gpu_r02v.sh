set -o pipefail
O=gpurun_out/r02v7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_aln.py tests/test_bwa_integration.py -m gpu -x -v --timeout 60 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/aln_prof.py --launches 2 --cycles $O/cyc.bin > $O/aln.log 2>&1 || exit 2
timeout -k 10 600 python -u tools/aln_prof.py --launches 2 --genome-profile human > $O/aln_human.log 2>&1 || exit 3
echo ALL OK
