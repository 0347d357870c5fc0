set -o pipefail
O=gpurun_out/r02al
mkdir -p $O /tmp/wc
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/aln_prof.py --launches 1 --lib gpurun_bisect/libsmemgpu_W.so --cycles /tmp/wc/u.bin > $O/u.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/aln_prof.py --launches 1 --genome-profile human --lib gpurun_bisect/libsmemgpu_W.so --cycles /tmp/wc/h.bin > $O/h.log 2>&1 || exit 2
python3 tools/walk_cycles.py /tmp/wc/u.bin /tmp/wc/h.bin > $O/walk.txt 2>&1 || exit 3
echo ALL OK
