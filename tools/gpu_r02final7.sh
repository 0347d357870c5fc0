# round-2 measurements after the chaining changes: every GPU test, traffic
# for this build, bench c2 (uniform and human-like), the rocprof summary, smoke
set -o pipefail
O=gpurun_out/${FINAL_OUT:-final7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/traffic.py --out $O/traffic.json --tmp $O/traffic > $O/traffic.log 2>&1 || exit 2
cp $O/traffic.json profiles/traffic.json
timeout -k 10 600 python -u bench.py --steps 10 > $O/bench_c2.json 2> $O/bench_c2.err || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 -- python3 -u bench.py --steps 10 --stream-reads -1 --parity 0 --side-stages 0 --cpu-seconds 0 > $O/prof_bench_c2.json 2> $O/prof_bench_c2.err || exit 4
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 5
timeout -k 10 900 python -u bench.py --steps 10 --genome-profile human > $O/bench_c2_human.json 2> $O/bench_c2_human.err || exit 6
echo ALL OK
