#!/bin/bash
# Round-2 probes: random-probe ceilings for interval tables of K = 13..16
# (mode 7) beside the Occ64 fetch (mode 6), FETCH_SIZE calibration on both
# shapes (known bytes vs counter), and the human-size extend profile.
set -o pipefail
OUT=${1:-gpurun_out/probe}
mkdir -p "$OUT"
export TMPDIR=/tmp
G=$(pwd)/bwa-mem-harp2_amd/bin/gather_ceiling
for mb in 3100 ; do timeout -k 10 60 "$G" $mb 12 2000 6 >> "$OUT/ceiling.jsonl" || exit 1; done
for mb in 1432 5728 22912 91648; do timeout -k 10 60 "$G" $mb 12 2000 7 >> "$OUT/ceiling.jsonl" || exit 1; done
for mb in 22912; do timeout -k 10 60 "$G" $mb 16 2000 7 >> "$OUT/ceiling.jsonl" || exit 1; done
echo ceilings ok
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gather --output-format csv -d "$OUT/fs6" -o p -- "$G" 3100 12 1000 6 > "$OUT/fs6.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gather --output-format csv -d "$OUT/fs7" -o p -- "$G" 22912 12 1000 7 > "$OUT/fs7.log" 2>&1 || exit 1
echo pmc ok
timeout -k 10 600 python -u tools/ext_profile.py --gpu --reads 20000 --threads 16 --out "$OUT/ext_profile_human.json" > "$OUT/ext_profile.log" 2>&1 || exit 1
echo profile ok
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex gather --output-format csv -d "$OUT/rq6" -o p -- "$G" 3100 12 1000 6 > "$OUT/rq6.log" 2>&1 || exit 1
echo rdreq ok
