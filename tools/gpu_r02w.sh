set -o pipefail
O=gpurun_out/r02w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest "tests/test_aln.py::test_aln_gpu_vs_reference" -m gpu -x -v -s --timeout 90 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo ALL OK
