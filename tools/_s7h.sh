# round-6 scratch driver: the raw-output capacity per read vs overflow reads (human-like c2 and c5)
mkdir -p gpurun_out/s7h
timeout -k 10 600 python -u tools/intv_cap_sweep.py --caps 48,56,64,80,0 > gpurun_out/s7h/cap_c2.jsonl 2> gpurun_out/s7h/cap_c2.err || { echo "c2 failed"; exit 1; }
timeout -k 10 600 python -u tools/intv_cap_sweep.py --caps 56,64,80,0 --config c5 > gpurun_out/s7h/cap_c5.jsonl 2> gpurun_out/s7h/cap_c5.err && echo "ALL OK s7h"
