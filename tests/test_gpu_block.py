"""GPU parity of the bloom-block path (lsmb_build_block):
the block bytes must equal BloomFilter::serialize of the oracle-built filter
(src/bloom/mod.rs:102-115) for fixed, var-length, empty and all-empty-key
batches, single- and multi-chunk (the H2D pipeline's two staging slots), and an
SSTable written with the GPU block must load into the device FilterSet and
answer like the oracle.
"""
import os

import numpy as np
import pytest

import keygen
import lsmbloom
from lsmbloom import sstable

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = lsmbloom.Context(0)
    yield c
    c.close()


@pytest.fixture
def small_chunks():
    old = os.environ.get("LSMB_H2D_CHUNK_MB")
    os.environ["LSMB_H2D_CHUNK_MB"] = "1"
    yield
    if old is None:
        del os.environ["LSMB_H2D_CHUNK_MB"]
    else:
        os.environ["LSMB_H2D_CHUNK_MB"] = old


@pytest.mark.parametrize("n,fpr_n", [(1, 1000), (1000, 1000), (200_000, 200_000), (300_000, 6_000_000)])
def test_block_fixed16_vs_oracle(ctx, oracle, n, fpr_n):
    nb, k = lsmbloom.params(fpr_n, 0.01)
    keys = keygen.key16(0x5EED0001, 0, n)
    got = ctx.build_block(keys, nb, k, key_len=16)
    ref = oracle.serialize(oracle.build_fixed(keys, 16, nb, k), nb, k)
    assert got.size == lsmbloom.serialized_size(nb)
    assert bytes(got) == bytes(ref)


def test_block_multichunk_fixed_and_var(ctx, oracle, small_chunks):
    # 1 MiB chunks: 3 M 16-B keys = 46 chunks through the two staging slots
    n = 3_000_000
    nb, k = lsmbloom.params(n, 0.01)
    keys = keygen.key16(0x5EED0001, 0, n)
    ref = oracle.serialize(oracle.build_fixed_mt(keys, 16, nb, k, 8), nb, k)
    assert bytes(ctx.build_block(keys, nb, k, key_len=16)) == bytes(ref)
    data, offs = keygen.varlen(200_000)
    nb2, k2 = lsmbloom.params(200_000, 0.01)
    ref2 = oracle.serialize(oracle.build_var(data, offs, nb2, k2), nb2, k2)
    assert bytes(ctx.build_block(data, nb2, k2, offsets=offs)) == bytes(ref2)
    # OR-accumulating host entry point over the same pipeline
    w = np.zeros(lsmbloom.num_words(nb2), dtype=np.uint64)
    w[5] = 0xF0F0
    ref_w = oracle.build_var(data, offs, nb2, k2, words=w.copy())
    assert np.array_equal(ctx.build_var(data, offs, nb2, k2, words=w), ref_w)


def test_block_var_edge_cases(ctx, oracle):
    nb, k = lsmbloom.params(1000, 0.01)
    # empty batch: the empty filter's block (new() + serialize)
    empty = ctx.build_block(np.zeros(0, np.uint8), nb, k, offsets=np.zeros(1, np.uint64))
    assert bytes(empty) == bytes(oracle.serialize(np.zeros(lsmbloom.num_words(nb), np.uint64), nb, k))
    # all-empty keys (fixed key_len 0 and var with zero lengths) = one insert of b""
    w = np.zeros(lsmbloom.num_words(nb), np.uint64)
    oracle.insert(w, nb, k, b"")
    ref = bytes(oracle.serialize(w, nb, k))
    assert bytes(ctx.build_block(np.zeros(0, np.uint8), nb, k, offsets=np.zeros(4, np.uint64))) == ref
    # ragged keys including a 5000-byte one
    keys = [b"", b"a", b"key_0001", bytes(range(256)) * 20, b"\xff" * 300]
    data, offs = keygen.pack(keys)
    ref = oracle.serialize(oracle.build_var(data, offs, nb, k), nb, k)
    assert bytes(ctx.build_block(data, nb, k, offsets=offs)) == bytes(ref)
    # too small a buffer is rejected (no partial write contract)
    with pytest.raises(ValueError):
        ctx.build_block(data, nb, k, offsets=offs, out=np.zeros(100, np.uint8))


def test_builder_build_serialized(ctx, oracle):
    b = lsmbloom.BloomFilterBuilder.new(1000, 0.01, ctx=ctx)
    for i in range(100):
        b.add_key(b"key_%05d" % i)
    blk = b.build_serialized()
    data, offs = keygen.ascii_keys("key_{:05d}", range(100))
    nb, k = lsmbloom.params(1000, 0.01)
    assert blk == bytes(oracle.serialize(oracle.build_var(data, offs, nb, k), nb, k))


def test_sstable_gpu_block_roundtrip_into_fset(ctx, oracle, tmp_path):
    """Flush-shaped: keys -> GPU bloom block -> SST file -> SSTable::open-style
    read -> device FilterSet -> batched get() checks (reader.rs:192-199)."""
    fs = lsmbloom.FilterSet(ctx)
    tables = []
    for t in range(3):
        arena = sstable.KeyArena()
        ks = [b"t%d_key_%06d" % (t, i) for i in range(1500)]
        for kk in ks:
            arena.add(kk)
        path = tmp_path / ("%d.sst" % t)
        ft = sstable.finish_sstable(path, b"D" * (100 + t), t, arena, sstable.encode_index_entry(ks[-1], 0, 100 + t),
                                    expected_keys=len(ks), ctx=ctx)
        assert ft.bloom_block_offset + ft.bloom_block_size <= ft.index_block_offset
        slot = sstable.load_filter(fs, path)
        tables.append((slot, ks))
    probe = [kk for _, ks in tables for kk in ks[::50]] + [b"t1_key_9999999", b"zzz", b"t0_key_000000x"]
    got = fs.probe_keys(probe)
    nb, k = lsmbloom.params(1500, 0.01)
    for i, key in enumerate(probe):
        for slot, ks in tables:
            lo, hi = ks[0], ks[-1]
            d, o = keygen.pack(ks)
            exp = lo <= key <= hi and oracle.may_contain(oracle.build_var(d, o, nb, k), nb, k, key)
            assert bool((int(got[i]) >> slot) & 1) == bool(exp), (key, slot)
    fs.close()


def test_gen_varlen_dev_matches_keygen_and_builds_like_oracle(ctx, oracle):
    import torch
    for first, n in ((0, 1000), (12345, 777)):
        d, o = ctx.gen_varlen_dev(n, first=first)
        hd, ho = keygen.varlen(n, first=first)
        assert np.array_equal(o.cpu().numpy().astype(np.uint64), ho)
        assert np.array_equal(d.cpu().numpy(), hd)
    # C4-shaped device build (partition strategy) vs the oracle
    n = 400_000
    d, o = ctx.gen_varlen_dev(n)
    nb, k = lsmbloom.params(50 * n, 0.01)
    w = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=d.device)
    ctx.build_var_dev(d, o, n, nb, k, w)
    torch.cuda.synchronize()
    hd, ho = keygen.varlen(n)
    assert np.array_equal(w.cpu().numpy().view(np.uint64), oracle.build_var(hd, ho, nb, k))


def test_hash_var_windows_giant_keys_unaligned(ctx, oracle):
    """k_hash_var edge cases on the partition path: keys longer than the 40 KiB
    LDS window (hashed from global memory), workgroups that need several window
    rounds, runs of empty keys, and a data pointer that is not 16-B aligned."""
    import torch
    rng = np.random.default_rng(7)
    lens = rng.integers(8, 257, size=300_000)
    lens[1000:1400] = 0                         # empty keys
    lens[5000] = 50_000                         # > window: global path
    lens[5001] = 70_001
    lens[9000:9256] = 3000                      # 768 KB in one workgroup: many rounds
    lens[-1] = 41_000
    offs = np.zeros(lens.size + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    data = keygen.stream_bytes(0xABCDEF, int(offs[-1]))
    n = lens.size
    nb, k = lsmbloom.params(20_000_000, 0.01)
    assert lsmbloom.build_strategy(nb, n) == "partition"
    ref = oracle.build_var(data, offs, nb, k)
    dev = torch.device("cuda:0")
    raw = torch.zeros(data.size + 64, dtype=torch.uint8, device=dev)
    raw[5:5 + data.size] = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    w = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    ctx.build_var_dev(raw[5:], d_offs, n, nb, k, w)
    torch.cuda.synchronize()
    assert np.array_equal(w.cpu().numpy().view(np.uint64), ref)
