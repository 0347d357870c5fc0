# Are the streaming leg's pinned copies SDMA transfers or blit kernels, and
# does HSA_ENABLE_SDMA change the PCIe-inclusive rate?
set -o pipefail
O=gpurun_out/sdma
mkdir -p $O
export TMPDIR=/tmp
(env | grep -iE "sdma|^hsa_|^hip_|^gpu_|^roc" || true) > $O/env.txt
B="bench.py --steps 3 --warmup 1 --parity 0 --side-stages 0 --cpu-seconds 0"
timeout -k 10 400 python -u $B > $O/default.json 2> $O/default.err || exit 1
HSA_ENABLE_SDMA=1 timeout -k 10 400 python -u $B > $O/sdma1.json 2> $O/sdma1.err || exit 2
HSA_ENABLE_SDMA=0 timeout -k 10 400 python -u $B > $O/sdma0.json 2> $O/sdma0.err || exit 3
HSA_ENABLE_SDMA=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof1 -o s1 -- python3 -u $B --stream-passes 1 > $O/prof1.json 2> $O/prof1.err || exit 4
echo ALL OK
