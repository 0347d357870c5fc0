# the default build vs every kernel file under max-ilp scheduling (abtest/ilpall), alternating
set -o pipefail
O=gpurun_out/flags2
mkdir -p $O
export TMPDIR=/tmp
for L in default ilpall default ilpall; do
  if [ $L = default ]; then LIB=bwa-mem-harp2_amd/lib/libsmemgpu.so; else LIB=abtest/$L/libsmemgpu.so; fi
  SMEMGPU_LIB=$PWD/$LIB timeout -k 10 400 python -u bench.py --steps 10 --stream-reads -1 --parity 0 --cpu-seconds 0 > $O/bench_$L.json.tmp 2>> $O/bench.err || exit 1
  (echo -n "$L "; cat $O/bench_$L.json.tmp) >> $O/bench.jsonl
done
echo ALL OK
