"""Multi-process (gloo, CPU) tests of the sharded-build merge (lsmbloom.dist).

A run's keys are split into contiguous shards, one per rank; each rank builds a
full-size partial filter over its shard (here with the CPU oracle: the GPU
build itself is covered by tests/test_gpu_parity.py) and the ranks merge the
partials with the bitwise-OR allreduce.  The merged words must equal the
single-process build of all keys, bit for bit, on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, nbits, k, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "storage-engine_amd"))
    sys.path.insert(0, here)
    import keygen
    import oracle_ct
    from lsmbloom import dist as ldist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = oracle_ct.load()
        lo, hi = n * rank // world, n * (rank + 1) // world
        part = orc.build_fixed(keygen.key16(0x5EED0001, lo, hi - lo), 16, nbits, k)
        words = torch.from_numpy(part.view(np.int64).copy())
        mine, start = ldist.or_reduce_scatter_(words.clone())
        ldist.or_allreduce_(words)
        q.put((rank, words.numpy().view(np.uint64).copy(), mine.numpy().view(np.uint64).copy(), start))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,nbits", [(2, 200_000, 1_917_011), (3, 150_001, 3_000_017),
                                           (2, 50_000, 64 * 1001), (2, 50_000, 64 * 1000),
                                           (4, 80_000, 64 * 4096)])
def test_sharded_build_or_allreduce(oracle, world, n, nbits):
    import keygen
    k = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, nbits, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = oracle.build_fixed(keygen.key16(0x5EED0001, 0, n), 16, nbits, k)
    slices = {}
    for rank, words, mine, start in res:
        assert np.array_equal(words, ref), "rank %d merged filter differs" % rank
        slices[rank] = (start, mine)
    # reduce-scatter: rank r holds words [start, start + len) of the merged filter
    for rank, (start, mine) in slices.items():
        end = min(start + mine.size, ref.size)
        assert np.array_equal(mine[: end - start], ref[start:end])
