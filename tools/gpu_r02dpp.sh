# fused DPP max scans in extend_wave; ksw_extend_kernel on the shared extend_wave
set -o pipefail
O=gpurun_out/dpp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ksw.py tests/test_aln.py tests/test_ksw_align.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 3 --stream-reads -1 --parity 0 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || exit 2
for P in uniform human; do
  echo "== $P" >> $O/aln.log
  timeout -k 10 500 python -u tools/aln_prof.py --launches 3 --genome-profile $P >> $O/aln.log 2>&1 || exit 3
done
echo ALL OK
