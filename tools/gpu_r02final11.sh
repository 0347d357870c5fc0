# per-kernel times of the chaining and alignment stages on the final build
set -o pipefail
O=gpurun_out/final11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/u -o u -- python3 -u tools/aln_prof.py --launches 1 > $O/u.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/h -o h -- python3 -u tools/aln_prof.py --launches 1 --genome-profile human > $O/h.log 2>&1 || exit 2
echo ALL OK
