# round-6 scratch driver: the intermittent eight-context failure, by setting
mkdir -p gpurun_out/s6j
timeout -k 10 900 python -u tools/flaky_probe.py --reps 6 --out gpurun_out/s6j/flaky.json > gpurun_out/s6j/flaky.log 2>&1 && echo "ALL OK s6j"
