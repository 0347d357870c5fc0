# round-6 scratch driver: per-read cycles of the alignment stage (the heavy walk's tail)
mkdir -p gpurun_out/s6g
timeout -k 10 600 python -u tools/aln_prof.py --launches 2 --cycles gpurun_out/s6g/cyc > gpurun_out/s6g/aln_cycles.log 2>&1 || { echo "aln cycles failed"; exit 1; }
echo "ALL OK s6g"
