#!/bin/bash
# Counter passes over the lane-per-problem ksw_extend2 kernel (tools/ksw_ab.py
# workload, problems with qlen <= 128), one rocprofv3 run per pass.
#   bash tools/pmc_ksw.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/pmc_ksw}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM"
)
for i in "${!PASSES[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc ${PASSES[$i]} --kernel-include-regex ksw_lane_kernel --output-format csv \
    -d "$OUT" -o pass$i -- python tools/ksw_ab.py --max-qlen 128 --reps 1 --problems 2000000 --only lane \
    > "$OUT/pass$i.log" 2>&1 \
    || { echo "pass $i failed rc=$?"; tail -5 "$OUT/pass$i.log"; exit 1; }
done
python tools/pmc_sum.py --by-kernel "$OUT" > "$OUT/sum.json"
echo "all passes ok"
