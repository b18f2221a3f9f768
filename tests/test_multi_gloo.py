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


def _range_worker(rank, world, port, n, nbits, k, ranges, q):
    """bench.py's overlapped N > 1 step on the CPU: the partial filter's sweep
    ranges are OR-allreduced one view at a time (or_allreduce_(words[a:b]))."""
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
        for a, b in ranges:
            v = words[a:b]
            ldist.or_allreduce_(v)
            assert v.data_ptr() == words[a:].data_ptr()  # merged in place, inside the view
        q.put((rank, words.numpy().view(np.uint64).copy()))
    finally:
        dist.destroy_process_group()


def test_slice_arithmetic_world8_c5_ranges():
    """The N = 8 C5 merge's slicing: each of C5's two
    2^25-word sweep ranges splits into 8 equal even slices, so the all-gather
    lands straight in the range's view (no staging copy), and the slices tile
    the range."""
    import lsmbloom
    from lsmbloom import dist as ldist
    nb, k = lsmbloom.params(1_000_000_000, 0.01)
    assert lsmbloom.build_sweeps(nb, 125_000_000, k) == 2
    rng = [lsmbloom.sweep_words(nb, 125_000_000, s, k) for s in range(2)]
    assert rng == [(0, 1 << 25), (1 << 25, 1 << 26)]
    for world in (2, 4, 8):
        for a, b in rng:
            per = ldist._slices(b - a, world)
            assert per * world == b - a and per % 2 == 0
    # ragged ranges fall back to a staged gather: slices still cover every word
    for n, world in [(1000, 8), (14_948_677, 8), (3, 8), (17, 3)]:
        per = ldist._slices(n, world)
        assert per % 2 == 0 and per * world >= n and (per - 2) * world < n


@pytest.mark.parametrize("world,R,tail", [(8, 1 << 14, 0), (8, 1 << 12, 1234)])
def test_world8_sweep_range_allreduce(oracle, world, R, tail):
    """8 gloo ranks merge a 2-sweep filter range by range, as bench.py's
    overlapped C5 step does (2^25-word ranges at full size; 2^14 here), plus a
    ragged last range: every rank ends with the single-process build."""
    import keygen
    k = 7
    nbits = 64 * (2 * R + tail)
    ranges = [(0, R), (R, 2 * R + tail)]
    n = 120_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_range_worker, args=(r, world, port, n, nbits, k, ranges, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = oracle.build_fixed(keygen.key16(0x5EED0001, 0, n), 16, nbits, k)
    for rank, words in res:
        assert np.array_equal(words, ref), "rank %d merged filter differs" % rank
