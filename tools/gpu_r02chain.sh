# chaining stage: per-phase cycles of the heaviest reads (SMEM_CHAIN_DBG)
set -o pipefail
O=gpurun_out/chain
mkdir -p $O
export TMPDIR=/tmp
for P in uniform human; do
  SMEM_CHAIN_DBG=1 timeout -k 10 500 python -u tools/chain_prof.py --genome-profile $P > $O/chain_$P.json 2> $O/chain_$P.err || exit 1
done
echo ALL OK
