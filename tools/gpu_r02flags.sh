# seed_kernel under other compiler scheduling strategies (abtest/<name>/libsmemgpu.so, SMEMGPU_LIB)
set -o pipefail
O=gpurun_out/flags
mkdir -p $O
export TMPDIR=/tmp
for L in default maxilp iterilp o2 default; do
  if [ $L = default ]; then LIB=bwa-mem-harp2_amd/lib/libsmemgpu.so; else LIB=abtest/$L/libsmemgpu.so; fi
  echo "== $L" >> $O/sweep.jsonl
  SMEMGPU_LIB=$PWD/$LIB timeout -k 10 300 python -u tools/sweep.py --genome-mbp 3101.804739 --lanes 768 --reps 5 --variants 2 >> $O/sweep.jsonl 2>> $O/sweep.err || exit 1
done
echo ALL OK
