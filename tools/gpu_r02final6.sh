set -o pipefail
O=gpurun_out/final6
mkdir -p $O
export TMPDIR=/tmp
for c in c3 c4 c5; do
  timeout -k 10 600 python -u bench.py --steps 10 --config $c --side-stages 0 > $O/bench_$c.json 2> $O/bench_$c.err || exit 2
done
timeout -k 10 900 python -u bench.py --steps 10 --genome-profile human > $O/bench_c2_human.json 2> $O/bench_c2_human.err || exit 3
echo ALL OK
