# Rehearse the driver's N>1 launch on a one-GPU box: two ranks on cuda:0
# (gloo, since RCCL refuses two ranks on one device); checks the multi-rank
# path end to end, the numbers are not a scaling measurement.
set -o pipefail
O=gpurun_out/rank2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err || exit 1
echo ALL OK
