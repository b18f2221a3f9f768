"""Streaming ingestion on the GPU (lsmb_stream).

Mirrors the flush loop: `for (key, value) in frozen.iter() { builder.add(key,
value) }` (src/db/mod.rs:379-383 -> SSTableBuilder::add ->
BloomFilterBuilder::add_key, src/sstable/builder.rs:93) and the compaction
loop over merged entries (src/compaction/scheduler.rs:152-158), with small
staging chunks so that many chunks are uploaded and built while keys are still
being added.  Every block / word array is compared with the oracle.
"""
import os

import numpy as np
import pytest

import keygen
import lsmbloom

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = lsmbloom.Context(0)
    yield c
    c.close()


@pytest.fixture
def small_chunks():
    old = os.environ.get("LSMB_STREAM_CHUNK_MB")
    os.environ["LSMB_STREAM_CHUNK_MB"] = "1"
    yield
    if old is None:
        del os.environ["LSMB_STREAM_CHUNK_MB"]
    else:
        os.environ["LSMB_STREAM_CHUNK_MB"] = old


def test_stream_memtable_walk_one_key_at_a_time(ctx, oracle, small_chunks):
    # a sorted memtable of var-len keys, walked in order, one add per key
    n = 200_000
    data, offs = keygen.varlen(n)
    keys = sorted(bytes(data[offs[i]:offs[i + 1]]) for i in range(n))
    nb, k = lsmbloom.params(n, 0.01)
    st = lsmbloom.KeyStream(ctx, nb, k)
    for key in keys:
        st.add(key)
    assert st.count() == n
    blk = st.finish_block()
    d, o = keygen.pack(keys)
    assert bytes(blk) == bytes(oracle.serialize(oracle.build_var(d, o, nb, k), nb, k))
    st.close()


@pytest.mark.parametrize("filter_n", [3_000_000, 40_000_000])  # tiled / partition builds per chunk
def test_stream_batches_many_chunks(ctx, oracle, small_chunks, filter_n):
    n = 3_000_000
    keys = keygen.key16(0x5EED0001, 0, n)
    nb, k = lsmbloom.params(filter_n, 0.01)
    st = lsmbloom.KeyStream(ctx, nb, k)
    flat = np.ascontiguousarray(keys).reshape(-1)
    step = 250_000  # iterator batches; a 1 MiB chunk holds 65 536 16-B keys
    for a in range(0, n, step):
        m = min(step, n - a)
        st.add_batch(flat[a * 16:(a + m) * 16], np.arange(m + 1, dtype=np.uint64) * 16)
    w = st.finish_words()
    assert np.array_equal(w, oracle.build_fixed_mt(keys, 16, nb, k, 8))
    st.close()


def test_stream_reuse_reset_and_threshold(ctx, oracle):
    # The gpu marker's fixture forces host_max_keys() = 0; a ctx-backed stream
    # must also cross a real threshold: at 64 keys the run finishes with the
    # host loop out of the pinned staging, at 65 it goes to the device
    # (ADVICE r02).
    nb, k = lsmbloom.params(50_000, 0.01)
    st = lsmbloom.KeyStream(ctx, nb, k)
    old = lsmbloom.host_max_keys()
    lsmbloom.set_host_max_keys(64)
    try:
        for rnd, n in enumerate((50_000, 100, 64, 65, 1, 0, 64)):
            keys = keygen.key16(0x1000 + rnd, 0, n) if n else np.zeros((0, 16), np.uint8)
            for i in range(n):
                st.add(bytes(keys[i]))
            w = st.finish_words()
            assert np.array_equal(w, oracle.build_fixed(keys, 16, nb, k)), (rnd, n)
    finally:
        lsmbloom.set_host_max_keys(old)
    nb2, k2 = lsmbloom.params(2_000_000, 0.001)
    st.reset(nb2, k2)
    keys = keygen.key16(7, 0, 300_000)
    flat = np.ascontiguousarray(keys).reshape(-1)
    st.add_batch(flat, np.arange(300_001, dtype=np.uint64) * 16)
    blk = st.finish_block()
    assert bytes(blk) == bytes(oracle.serialize(oracle.build_fixed(keys, 16, nb2, k2), nb2, k2))
    st.close()


def test_flush_e2e_tool():
    """The C++ flush-shaped end-to-end driver (tools/flush_e2e.cpp): memtable
    walk -> lsmb_stream -> serialized block, bit-identical to the per-key host
    insert loop (the reference's flush) on the same keys."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "storage-engine_amd", "build", "flush_e2e")
    r = subprocess.run([exe, "300000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["bit_exact"] is True and out["keys"] == 300000
