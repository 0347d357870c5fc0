# round-6 scratch driver: c4 / c5 streaming -- smaller chunks, more workers
mkdir -p gpurun_out/s7a
timeout -k 10 600 python -u tools/stream_sweep.py --config c5 --chunks 524288,786432,1048576 --workers 4,6,8 > gpurun_out/s7a/stream_c5.jsonl 2> gpurun_out/s7a/stream_c5.err || { echo "c5 sweep failed"; exit 1; }
timeout -k 10 600 python -u tools/stream_sweep.py --config c4 --chunks 524288,1048576 --workers 4,6,8 > gpurun_out/s7a/stream_c4.jsonl 2> gpurun_out/s7a/stream_c4.err && echo "ALL OK s7a"
