set -o pipefail
mkdir -p gpurun_out/r02l
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/prof_run.py --launches 2 > gpurun_out/r02l/warm.log 2>&1 || exit 1
for spec in "2 0" "23 8" "23 12" "11 0" "16 0"; do
  set -- $spec
  PMC_PASSES="1 2" timeout -k 10 600 bash tools/pmc_passes.sh gpurun_out/r02l/v$1_k$2 --variant $1 --kmer-k $2 --launches 2 > gpurun_out/r02l/v$1_k$2.log 2>&1 || exit 2
done
echo ALL OK
