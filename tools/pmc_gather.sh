#!/bin/bash
# Counter passes over tools/gather_ceiling.hip modes (random 64-B buckets).
# Usage: tools/pmc_gather.sh <outdir> <mode...>
set -o pipefail
OUT=${1:-gpurun_out/pmcg}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
G=$(pwd)/bwa-mem-harp2_amd/bin/gather_ceiling
PASSES=(
  "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM"
  "TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_MISS TCP_TCC_READ_REQ_LATENCY TD_TD_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES"
  "TA_TA_BUSY TA_TOTAL_WAVEFRONTS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES"
)
for m in "$@"; do
  i=0
  for P in "${PASSES[@]}"; do
    timeout -k 10 120 rocprofv3 --pmc $P --kernel-include-regex gather --output-format csv -d "$OUT/m$m" -o pass$i -- "$G" 1000 12 1000 "$m" > "$OUT/m$m.pass$i.log" 2>&1 || { echo "mode $m pass $i failed"; exit 1; }
    i=$((i+1))
  done
done
echo "all passes ok"
