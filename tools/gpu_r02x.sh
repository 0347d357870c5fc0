set -o pipefail
O=gpurun_out/r02x
mkdir -p $O
export TMPDIR=/tmp
SMEM_ALN_HEAVY_MIN=0 timeout -k 10 100 python -u -m pytest "tests/test_aln.py::test_aln_gpu_vs_reference" -m gpu -x -q -k "default and g1_default" --timeout 60 --timeout-method thread > $O/t_heavy0.log 2>&1; echo "heavy0 rc=$?" >> $O/rc.txt
AMD_LOG_LEVEL=3 timeout -k 10 100 python -u -m pytest "tests/test_aln.py::test_aln_gpu_vs_reference" -m gpu -x -q -k "default and g1_default" --timeout 60 --timeout-method thread > $O/t_log.log 2>&1; echo "log rc=$?" >> $O/rc.txt
echo ALL DONE
