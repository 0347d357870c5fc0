#!/bin/bash
# One gpurun call = a list of named steps, each under its own time limit,
# stopping at the first failure (no GPU step runs after a failed one):
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh <out> <step> [<step> ...]'
#
# Outputs land in gpurun_out/<out>/.  Steps (ARGS: bench.py / tool arguments
# with commas for spaces, e.g. bench:--steps,10,--genome-profile,human):
#   tests[:FILTER]    python -m pytest tests -m gpu [-k FILTER] (commas: spaces, e.g. tests:product,or,variants) -> tests.log
#   smoke             __graft_entry__.smoke()                         -> smoke.log
#   traffic[:ARGS]    tools/traffic.py for this build (TCC_EA0_RDREQ per launch) -> traffic.json,
#                     copied to profiles/traffic_human.json (the default human-like workload) or, with
#                     --genome-profile,uniform, profiles/traffic.json
#   bench[:ARGS]      python bench.py ARGS                           -> bench<k>.json / .err
#   rocprof[:ARGS]    rocprofv3 --kernel-trace --stats over bench.py's timed seeding steps -> prof<k>/
#   pmc:PASSES[:ARGS] tools/pmc_passes.sh, passes "1,2" of its list, ARGS for tools/prof_run.py (bench workload
#                     args, --variant, --launches) -> pmc<k>/
#   stamps[:ARGS]     tools/stamps.py (variant-9 cycle split)        -> stamps<k>.log
#   aln[:ARGS] / chain[:ARGS]   tools/aln_prof.py / tools/chain_prof.py under rocprofv3 --kernel-trace --stats
#   py:SCRIPT[:ARGS]  python SCRIPT ARGS                              -> py<k>.log
#   dist2[:ARGS]      bench.py --gpus 2 ARGS under torch.distributed.run, two ranks (on a one-GPU box both
#                     share cuda:0 over gloo: the driver's N>1 launch line rehearsed) -> dist2_<k>.json / .err
#   env:VAR=v[,VAR=v] exported for the steps after it (e.g. env:PMC_PROG=tools/aln_prof.py,PMC_KERNEL=aln_kernel)
# Replaces round 2's one-off tools/gpu_r02*.sh scripts (their outputs are under profiles/r02/).
set -o pipefail
OUT=gpurun_out/${1:?usage: gpu_run.sh <out> <step>...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
k=0
for step in "$@"; do
  k=$((k + 1))
  name=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  args=${arg//,/ }
  echo "[gpu_run] step $k: $step" >&2
  case "$name" in
    tests)
      sel=()
      [ -n "$arg" ] && sel=(-k "$args")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" \
        > "$OUT/tests.log" 2>&1 || { echo "tests failed"; exit $k; } ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { echo "smoke failed"; exit $k; } ;;
    traffic)
      timeout -k 10 600 python -u tools/traffic.py --out "$OUT/traffic$k.json" --tmp "$OUT/traffic$k" $args \
        > "$OUT/traffic$k.log" 2>&1 || { echo "traffic failed"; exit $k; }
      prof=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['workload']['genome_profile'])" "$OUT/traffic$k.json")
      if [ "$prof" = human ]; then cp "$OUT/traffic$k.json" profiles/traffic_human.json
      else cp "$OUT/traffic$k.json" profiles/traffic.json; fi ;;
    bench)
      timeout -k 10 1000 python -u bench.py $args > "$OUT/bench$k.json" 2> "$OUT/bench$k.err" \
        || { echo "bench failed"; tail -5 "$OUT/bench$k.err"; exit $k; } ;;
    rocprof)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$k" -o run -- \
        python3 -u bench.py --stream-reads -1 --parity 0 --side-stages 0 --cpu-seconds 0 --e2e-reads 0 --other-profile 0 \
        $args > "$OUT/prof$k.json" 2> "$OUT/prof$k.err" || { echo "rocprof failed"; exit $k; } ;;
    pmc)
      passes=${arg%%:*}
      rest=""
      [[ "$arg" == *:* ]] && rest=${arg#*:}
      PMC_PASSES="${passes//,/ }" timeout -k 10 900 bash tools/pmc_passes.sh "$OUT/pmc$k" ${rest//,/ } \
        > "$OUT/pmc$k.log" 2>&1 || { echo "pmc failed"; exit $k; } ;;
    stamps)
      timeout -k 10 600 python -u tools/stamps.py $args > "$OUT/stamps$k.log" 2>&1 || { echo "stamps failed"; exit $k; } ;;
    aln|chain)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name$k" -o run -- \
        python3 -u tools/${name}_prof.py $args > "$OUT/$name$k.log" 2>&1 || { echo "$name failed"; exit $k; } ;;
    dist2)
      timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 $args > "$OUT/dist2_$k.json" 2> "$OUT/dist2_$k.err" \
        || { echo "dist2 failed"; tail -5 "$OUT/dist2_$k.err"; exit $k; } ;;
    env)
      export $args ;;
    py)
      script=${arg%%:*}
      rest=""
      [[ "$arg" == *:* ]] && rest=${arg#*:}
      timeout -k 10 900 python -u "$script" ${rest//,/ } > "$OUT/py$k.log" 2>&1 || { echo "py $script failed"; exit $k; } ;;
    *)
      echo "unknown step $step"; exit 99 ;;
  esac
done
echo "ALL OK"
