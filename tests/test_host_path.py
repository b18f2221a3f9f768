"""The size-bounded host path (SURVEY §7 hard-part 8).

SSTableBuilder::new always sizes the filter for 1 000 keys
(src/sstable/builder.rs:51,74) and adds keys one at a time
(src/bloom/builder.rs:21-23).  For builds that small a device round trip costs
more than the whole loop, so builds of at most lsmb_host_max_keys() keys run
the library's own host loop (the same xxh3 / exact-modulo code the kernels run,
compiled for the host) — never the oracle — and need no GPU and no context.
These tests run on the CPU; tests/test_multi_gpu.py checks the GPU side of the
threshold gives the same bits.
"""
import numpy as np
import pytest

import keygen
import lsmbloom
from lsmbloom import BloomFilter, BloomFilterBuilder


@pytest.fixture
def threshold():
    old = lsmbloom.host_max_keys()
    yield old
    lsmbloom.set_host_max_keys(old)


def test_default_threshold_covers_sst_sizing(threshold):
    # the reference's default SST sizing (1 000 keys) stays on the host
    assert threshold >= 1000


def test_builder_1000_keys_without_gpu(oracle, threshold):
    # SSTableBuilder::new -> BloomFilterBuilder::new(1000, 0.01) (builder.rs:74)
    b = BloomFilterBuilder.new(1000, 0.01)
    keys = [b"key_%05d" % i for i in range(1000)]
    for key in keys:
        b.add_key(key)
    bf = b.build()
    data, offs = keygen.pack(keys)
    ref = oracle.build_var(data, offs, bf.num_bits(), bf.num_hashes())
    assert np.array_equal(bf.bits, ref)
    assert all(bf.may_contain(key) for key in keys)


def test_builder_build_serialized_without_gpu(oracle, threshold):
    b = BloomFilterBuilder.new(1000, 0.01)
    keys = [b"exist_%06d" % i for i in range(700)] + [b""] + [bytes(range(256))]
    for key in keys:
        b.add_key(key)
    blk = b.build_serialized()
    data, offs = keygen.pack(keys)
    nb, k = lsmbloom.params(1000, 0.01)
    assert blk == bytes(oracle.serialize(oracle.build_var(data, offs, nb, k), nb, k))
    # the empty builder: BloomFilter::new(..).serialize()
    assert BloomFilterBuilder.new(1000, 0.01).build_serialized() == BloomFilter.new(1000, 0.01).serialize()


@pytest.mark.parametrize("key_len", [0, 1, 16, 33])
def test_block_fixed_len_host(oracle, threshold, key_len):
    n = 1500
    keys = bytes(keygen.stream_bytes(0xABC + key_len, n * key_len))
    nb, k = lsmbloom.params(n, 0.01)
    out = np.empty(lsmbloom.serialized_size(nb), dtype=np.uint8)
    a = np.frombuffer(keys, dtype=np.uint8) if len(keys) else np.zeros(1, np.uint8)
    lib = lsmbloom.lib()
    rc = lib.lsmb_build_block(None, lsmbloom._p(a, lsmbloom.u8p), None, key_len, n, nb, k,
                              lsmbloom._p(out, lsmbloom.u8p), out.size)
    assert rc == 0, lib.lsmb_last_error()
    if key_len:
        ref_w = oracle.build_fixed(np.frombuffer(keys, np.uint8).reshape(n, key_len), key_len, nb, k)
    else:  # n empty keys == one insert of b""
        ref_w = oracle.build_var(b"", np.zeros(2, np.uint64), nb, k)
    assert bytes(out) == bytes(oracle.serialize(ref_w, nb, k))


def test_threshold_boundary_needs_context_above(oracle, threshold):
    # at the threshold: host loop, no context; one key above: the GPU context
    # is required, and a NULL context is refused (never a silent host build)
    lsmbloom.set_host_max_keys(64)
    assert lsmbloom.host_max_keys() == 64
    nb, k = lsmbloom.params(64, 0.01)
    keys = keygen.key16(0x5EED0001, 0, 65)
    words = np.zeros(lsmbloom.num_words(nb), np.uint64)
    lib = lsmbloom.lib()
    a = np.ascontiguousarray(keys).reshape(-1)
    assert lib.lsmb_build_fixed(None, lsmbloom._p(a, lsmbloom.u8p), 16, 64, nb, k,
                                lsmbloom._p(words, lsmbloom.u64p)) == 0
    assert np.array_equal(words, oracle.build_fixed(keys[:64], 16, nb, k))
    assert lib.lsmb_build_fixed(None, lsmbloom._p(a, lsmbloom.u8p), 16, 65, nb, k,
                                lsmbloom._p(words, lsmbloom.u64p)) == lsmbloom.LSMB_EINVAL
    assert b"null ctx" in lib.lsmb_last_error()
    lsmbloom.set_host_max_keys(0)
    assert lsmbloom.host_max_keys() == 0


def test_host_path_or_accumulates(oracle, threshold):
    # builds OR into existing words (insert() after build(), shard merges)
    nb, k = lsmbloom.params(1000, 0.01)
    a = keygen.key16(1, 0, 500)
    b = keygen.key16(2, 0, 500)
    w = np.zeros(lsmbloom.num_words(nb), np.uint64)
    lib = lsmbloom.lib()
    for keys in (a, b):
        x = np.ascontiguousarray(keys).reshape(-1)
        assert lib.lsmb_build_fixed(None, lsmbloom._p(x, lsmbloom.u8p), 16, 500, nb, k,
                                    lsmbloom._p(w, lsmbloom.u64p)) == 0
    ref = oracle.build_fixed(b, 16, nb, k, words=oracle.build_fixed(a, 16, nb, k))
    assert np.array_equal(w, ref)


def test_stream_host_only_flush_loop(oracle, threshold):
    """lsmb_stream without a device context: the flush's add_key loop over a
    memtable-sized run (src/db/mod.rs:379-383, SSTableBuilder::new sizing)
    finishes on the host; a run past the threshold is refused, not built on
    the CPU."""
    nb, k = lsmbloom.params(1000, 0.01)
    st = lsmbloom.KeyStream(None, nb, k)
    memtable = sorted({b"key_%05d" % i: b"v" for i in range(1000)}.items())  # frozen.iter() order
    for key, _value in memtable:
        st.add(key)
    assert st.count() == 1000
    blk = st.finish_block()
    data, offs = keygen.pack([kv[0] for kv in memtable])
    assert bytes(blk) == bytes(oracle.serialize(oracle.build_var(data, offs, nb, k), nb, k))
    # the stream restarts empty: a second run of other keys
    for i in range(10):
        st.add(b"other_%d" % i)
    w = st.finish_words()
    d2, o2 = keygen.pack([b"other_%d" % i for i in range(10)])
    assert np.array_equal(w, oracle.build_var(d2, o2, nb, k))
    lsmbloom.set_host_max_keys(5)
    for i in range(6):
        st.add(b"k%d" % i)
    with pytest.raises(ValueError):
        st.finish_block()
    st.close()
