set -o pipefail
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
for c in c4 c5 c3; do
  timeout -k 10 500 python -u bench.py --steps 10 --config $c --side-stages 0 --cpu-seconds 10 > gpurun_out/r02h/bench_$c.json 2> gpurun_out/r02h/bench_$c.err || exit 1
done
echo ALL OK
