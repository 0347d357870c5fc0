set -o pipefail
O=gpurun_out/r02at
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ksw.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "
import sys, time; sys.path.insert(0,'bwa-mem-harp2_amd'); sys.path.insert(0,'.')
import os, numpy as np, smemgpu
from smemgpu import synth
g = synth.make_genome(2_000_000, seed=5, n_chrom=1)
idx = smemgpu.Index.build_gpu(g.codes)
gpu = smemgpu.Gpu(idx, device=0)
for mq in (255, 130, 75, 40):
    b = synth.make_ksw_tasks(g.codes, 200000, seed=7, max_qlen=mq)
    res = {}
    for mode in ('0','1','0','1'):
        os.environ['SMEM_KSW_G16'] = mode
        got, ms = gpu.ksw_extend(b)
        res.setdefault(mode, []).append(ms)
        if mode == '1': assert (got == res['g0']).all() if 'g0' in res else True
        res['g' + mode] = got
    print('max_qlen', mq, 'wave', round(min(res['0']),3), 'g16', round(min(res['1']),3), 'same', bool((res['g0']==res['g1']).all()), flush=True)
" > $O/time.log 2>&1 || exit 2
echo ALL OK
