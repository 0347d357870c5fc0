"""Multi-rank plumbing of bench.py on CPU (gloo, world_size 2).

The seeding path shards reads across GPUs with the index replicated and no
collective in the data path; the only cross-rank traffic is
the barrier around the timed region and the two scalar reductions of the
report.  This checks them with two real processes: shards are disjoint,
throughput is all ranks' reads over the slowest rank's time.
"""
import argparse
import json
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank: int, world: int, port: int, out_dir: str):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
    import bench
    from smemgpu import synth
    d = bench.Dist("gloo")
    args = argparse.Namespace(reads=300, read_len=150, seed=1, sub=0.02, genome_mbp=0.2)
    g = synth.make_genome(200_000, seed=1, n_chrom=2).codes
    reads = bench.make_reads(args, d.rank, g)
    d.barrier()
    value, emax = bench.aggregate(d, elapsed=1.0 + d.rank, reads_per_rank=reads.n, steps=3)
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as fh:
        json.dump({"value": value, "emax": emax, "n": int(reads.n),
                   "digest": int(np.bitwise_xor.reduce(reads.codes.view(np.uint8)[: (reads.codes.size // 8) * 8]
                                                       .view(np.uint64)))}, fh)
    d.close()


def test_two_rank_gloo(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [json.load(open(tmp_path / f"r{i}.json")) for i in range(world)]
    assert r[0]["n"] == r[1]["n"] == 300
    assert r[0]["digest"] != r[1]["digest"], "ranks must seed different read shards"
    for x in r:
        assert x["emax"] == pytest.approx(2.0)                 # slowest rank's time
        assert x["value"] == pytest.approx(2 * 300 * 3 / 2.0)  # all ranks' reads / max time
