#!/bin/bash
# Random 32-B Occ64-bucket request ceiling on the 3.1 GB human-size table, swept over occupancy
# (waves per CU) and memory-level parallelism (buckets per lane per round): tools/gather_ceiling.hip
# mode 8 (registers, no LDS: the asked occupancy is the one run).  One JSON line per run.
#   bash tools/ceiling_sweep.sh > out.jsonl
set -o pipefail
EXE=${EXE:-tools/bin/gather_ceiling}
for w in 8 12 16 24 32; do
  for nb in 1 2 4 8 16; do
    timeout -k 5 60 $EXE 3101 $w 1000 8 0 $nb || exit 1
  done
done
