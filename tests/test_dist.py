"""Multi-rank plumbing of bench.py on CPU (gloo, world_size 2).

The seeding path shards reads across GPUs with the index replicated and no
collective in the data path: the read stream is cut into
blocks dealt round-robin to the ranks; the only cross-rank traffic is the
barrier around the timed region and the two scalar reductions of the report.
This checks them with two real processes: shards are disjoint, reassembled in
block order they are exactly the single-rank stream of the same total, their
seeding results (through the C restatement) reassemble to the single-rank
results, and throughput is all ranks' reads over the slowest rank's time.
"""
import argparse
import json
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCK = 100


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _args(reads: int):
    return argparse.Namespace(reads=reads, read_len=150, seed=1, sub=0.02, genome_mbp=0.2, block=BLOCK, pairs=False)


def _genome():
    from smemgpu import synth
    return synth.make_genome(200_000, seed=1, n_chrom=2).codes


def _rank_main(rank: int, world: int, port: int, out_dir: str):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
    import bench
    d = bench.Dist("gloo")
    reads = bench.make_reads(_args(300), d.rank, _genome(), world)
    d.barrier()
    value, emax = bench.aggregate(d, elapsed=1.0 + d.rank, reads_per_rank=reads.n, steps=3)
    np.save(os.path.join(out_dir, f"codes{rank}.npy"), reads.codes)
    np.save(os.path.join(out_dir, f"offs{rank}.npy"), reads.offs)
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as fh:
        json.dump({"value": value, "emax": emax, "n": int(reads.n)}, fh)
    d.close()


def test_two_rank_gloo(tmp_path):
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    import bench
    from smemgpu import synth
    from oracle import oracle
    import smemgpu
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [json.load(open(tmp_path / f"r{i}.json")) for i in range(world)]
    assert r[0]["n"] == r[1]["n"] == 300
    for x in r:
        assert x["emax"] == pytest.approx(2.0)                 # slowest rank's time
        assert x["value"] == pytest.approx(2 * 300 * 3 / 2.0)  # all ranks' reads / max time
    shards = [synth.Reads(np.diff(np.load(tmp_path / f"offs{i}.npy")).astype(np.int32),
                          np.load(tmp_path / f"codes{i}.npy"), np.load(tmp_path / f"offs{i}.npy")) for i in range(world)]
    # reassembled in block order (block b on rank b % world) == the single-rank stream
    g = _genome()
    single = bench.make_reads(_args(600), 0, g, 1)
    order = []
    for b in range(600 // BLOCK):
        order.append(shards[b % world].subset(np.arange((b // world) * BLOCK, (b // world + 1) * BLOCK)))
    joined = synth.concat_reads(order)
    assert np.array_equal(joined.codes, single.codes) and np.array_equal(joined.offs, single.offs)
    assert not np.array_equal(shards[0].codes, shards[1].codes)
    # the seeding results of the shards reassemble to the single-rank results
    idx = smemgpu.Index.build(g)
    oi = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    try:
        want = synth.read_smgo(oracle.seed(oi, single.codes, single.offs, threads=4)[0])
        per = [synth.read_smgo(oracle.seed(oi, s.codes, s.offs, threads=4)[0]) for s in shards]
        got = []
        for b in range(600 // BLOCK):
            got.extend(per[b % world][(b // world) * BLOCK:(b // world + 1) * BLOCK])
        assert len(got) == len(want)
        assert all(len(x) == len(y) and all(np.array_equal(u, v) for u, v in zip(x, y)) for x, y in zip(got, want))
    finally:
        oi.close()


def test_pairs_geometry():
    """make_pairs: FR mates of one fragment, interleaved (software/bwamem.c:1600-1609)."""
    from smemgpu import synth
    g = _genome()
    reads, frag = synth.make_pairs(g, 400, 100, seed=5, sub_rate=0.0, n_rate=0.0, with_pos=True)
    assert reads.n == 800
    for k in range(400):
        p, ins, rc = (int(v) for v in frag[k])
        assert 100 <= ins
        a = g[p:p + 100]
        b = (3 - g[p + ins - 100:p + ins])[::-1]
        m1, m2 = reads.read(2 * k), reads.read(2 * k + 1)
        if rc:
            a, b = b, a
        assert np.array_equal(m1, a) and np.array_equal(m2, b)
    ins = frag[:, 1]
    assert 450 < ins.mean() < 550


def test_shard_blocks():
    import bench
    assert bench.shard_blocks(1_000_000, 0, 1) == [0, 1, 2, 3]
    assert bench.shard_blocks(1_000_000, 3, 8) == [3, 11, 19, 27]


def test_span_union():
    """bench.py's kernel busy time: the union of overlapping launch spans."""
    import bench
    assert bench.span_union([]) == 0
    assert bench.span_union([(5, 9)]) == 4
    assert bench.span_union([(0, 10), (5, 12), (20, 25), (21, 22)]) == 17
    assert bench.span_union([(20, 25), (0, 10), (10, 11)]) == 16
