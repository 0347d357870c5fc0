# round-6 scratch driver: c4 / c5 streaming -- 256k / 512k chunks, repeated
mkdir -p gpurun_out/s7b
timeout -k 10 600 python -u tools/stream_sweep.py --config c5 --chunks 262144,524288 --workers 4,8,4,8 > gpurun_out/s7b/stream_c5.jsonl 2> gpurun_out/s7b/stream_c5.err || { echo "c5 sweep failed"; exit 1; }
timeout -k 10 600 python -u tools/stream_sweep.py --config c4 --chunks 262144,524288 --workers 4,8,4,8 > gpurun_out/s7b/stream_c4.jsonl 2> gpurun_out/s7b/stream_c4.err && echo "ALL OK s7b"
