set -o pipefail
O=gpurun_out/r02u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/aln_prof.py --launches 2 --cycles $O/cyc.bin > $O/aln.log 2>&1 || exit 1
echo ALL OK
