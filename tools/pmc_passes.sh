#!/bin/bash
# Counter passes for the seeding kernel (one rocprofv3 run per pass; no trace
# domains combined with --pmc).  Usage: tools/pmc_passes.sh <outdir> [prof_run args]
# PMC_PROG / PMC_KERNEL select another workload / kernel (e.g. tools/aln_prof.py, aln_kernel).
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "FETCH_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS TA_TA_BUSY TA_TOTAL_WAVEFRONTS"
  "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM"
  "TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_MISS TCP_TCC_READ_REQ_LATENCY TD_TD_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES"
  "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU"
)
SEL=${PMC_PASSES:-$(seq 0 $((${#PASSES[@]} - 1)))}  # e.g. PMC_PASSES="0 1 2"
for i in $SEL; do
  P=${PASSES[$i]}
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-include-regex ${PMC_KERNEL:-'seed_(wp_)?kernel'} --output-format csv -d "$OUT" -o pass$i -- python ${PMC_PROG:-tools/prof_run.py} "$@" > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo "all passes ok"
