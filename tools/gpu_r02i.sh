set -o pipefail
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --steps 10 --genome-profile human > gpurun_out/r02i/bench_c2_human.json 2> gpurun_out/r02i/bench_c2_human.err || exit 1
timeout -k 10 600 python -u tools/ext_profile.py --gpu --reads 20000 --threads 16 --out gpurun_out/r02i/ext_profile_uniform.json > gpurun_out/r02i/ext_profile.log 2>&1 || exit 2
echo ALL OK
