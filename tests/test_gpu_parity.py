"""GPU parity: the HIP build/probe path (through the C ABI) vs the CPU oracle.

Bit-exact for every word of every filter and every probe answer.  Small cases
compare against the committed golden fixtures; larger ones against the oracle
(oracle/liboracle.so, the checker) on the same seeded inputs, up to the full
BASELINE C2 size (100 M keys) where the multi-threaded oracle finishes in seconds.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import keygen
import lsmbloom
from lsmbloom import BloomFilter, BloomFilterBuilder

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
KATS = json.load(open(os.path.join(GOLD, "bloom_kats.json")))
C1 = json.load(open(os.path.join(GOLD, "c1_fixture.json")))
VAR = json.load(open(os.path.join(GOLD, "varlen_fixture.json")))
FULL = json.load(open(os.path.join(GOLD, "fullsize_fixture.json")))  # tests/golden/gen_fullsize.py


def assert_full_fixture(host_words, name):
    """The GPU's full-size filter == the oracle's (digest committed in
    tests/golden/fullsize_fixture.json): popcount, first/last words, sha256."""
    import hashlib
    fx = FULL[name]
    w = np.ascontiguousarray(host_words, dtype="<u8")
    assert w.size == fx["words"]
    assert [int(x) for x in w[:8]] == fx["first8"] and [int(x) for x in w[-8:]] == fx["last8"], name
    assert int(np.bitwise_count(w).sum()) == fx["popcount"], name
    assert hashlib.sha256(w.tobytes()).hexdigest() == fx["sha256"], name


@pytest.fixture(scope="module")
def ctx():
    c = lsmbloom.Context(0)
    yield c
    c.close()


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def ser(words, nb, k):
    f = BloomFilter(words, k, nb)
    return f.serialize()


# ---------------------------------------------------------------- golden fixtures
def test_c1_fixture_gpu(ctx):
    keys = keygen.key16(0x5EED0001, 0, C1["n"])
    nb, k = lsmbloom.params(C1["n"], 0.01)
    assert lsmbloom.build_strategy(nb, C1["n"]) == "lds"
    w = ctx.build_fixed(keys, 16, nb, k)
    assert sha(ser(w, nb, k)) == C1["serialized_sha256"]
    nm = keygen.key16(0x5EED0002, 0, C1["n"])
    m = ctx.probe([(w, nb, k)], nm, key_len=16)
    assert int(m.sum()) == C1["nonmember_false_positives"]
    assert sha(m.reshape(-1)) == C1["nonmember_probe_sha256"]
    assert ctx.probe([(w, nb, k)], keys, key_len=16).all()  # no false negatives


def test_reference_scenarios_gpu_builder(ctx):
    for sc in KATS["scenarios"]:
        b = BloomFilterBuilder.new(sc["n"], sc["fpr"], ctx=ctx)
        for key in sc["inserts"]:
            b.add_key(bytes.fromhex(key))
        bf = b.build()
        assert sha(bf.serialize()) == sc["serialized_sha256"], sc["name"]
        probes = [bytes.fromhex(p[0]) for p in sc["probes"]]
        m = BloomFilter.may_contain_batch([bf], probes, ctx=ctx)
        assert [bool(x) for x in m[:, 0]] == [p[1] for p in sc["probes"]], sc["name"]


def test_reference_fpr_counts_gpu(ctx):
    from test_oracle_golden import _fmt_keys
    for c in KATS["counts"]:
        ins, probes = _fmt_keys(c)
        nb, k = lsmbloom.params(c["n"], c["fpr"])
        d, o = keygen.pack(ins)
        w = ctx.build_var(d, o, nb, k)
        assert sha(ser(w, nb, k)) == c["serialized_sha256"], c["name"]
        pd, po = keygen.pack(probes)
        m = ctx.probe([(w, nb, k)], pd, po)
        if "false_positives" in c:
            assert int(m.sum()) == c["false_positives"], c["name"]


def test_varlen_fixture_gpu(ctx):
    data, offs = keygen.varlen(VAR["n"])
    nb, k = lsmbloom.params(VAR["n"], 0.01)
    w = ctx.build_var(data, offs, nb, k)
    assert sha(ser(w, nb, k)) == VAR["serialized_sha256"]
    nm = keygen.key16(0x5EED0002, 0, VAR["n"])
    assert int(ctx.probe([(w, nb, k)], nm, key_len=16).sum()) == VAR["nonmember_false_positives"]


# ---------------------------------------------------------------- oracle parity
def _cmp(a, b):
    assert a.shape == b.shape
    bad = np.nonzero(a != b)[0]
    assert bad.size == 0, "first mismatching words: %s" % bad[:8]


@pytest.mark.parametrize("n,fpr", [(1, 0.01), (1000, 0.01), (70_000, 0.001), (300_000, 0.01),
                                   (2_000_001, 0.01), (5_000_000, 0.05), (7_000_000, 0.01),
                                   (12_345_678, 0.001)])
def test_build_fixed16_vs_oracle(ctx, oracle, n, fpr):
    keys = keygen.key16(0x5EED0001, 0, n)
    nb, k = lsmbloom.params(n, fpr)
    _cmp(ctx.build_fixed(keys, 16, nb, k), oracle.build_fixed(keys, 16, nb, k))


def test_build_partition_huge_filter(ctx, oracle):
    # the C5 filter: new(1e9, 0.01) saturates to 2^32-1 bits (mod.rs:49), 512 MiB
    n = 3_000_000
    nb, k = lsmbloom.params(10**9, 0.01)
    assert nb == 2**32 - 1
    keys = keygen.key16(0x5EED0001, 0, n)
    assert lsmbloom.build_strategy(nb, n) == "partition"
    w = ctx.build_fixed(keys, 16, nb, k)
    ref = oracle.build_fixed_mt(keys, 16, nb, k, 16)
    _cmp(w, ref)
    # probe against the 2^32-1-bit filter: the bit-sliced table sizing once
    # wrapped at 32 bits here (nb + 31) and answered 0 for every key
    q = np.concatenate([keys[:50_000], keygen.key16(0x5EED0002, 0, 50_000)])
    for nf in (1, 3):
        got = ctx.probe([(w, nb, k)] * nf, q, key_len=16)
        exp = oracle.probe([(ref, nb, k)] * nf, q, key_len=16)
        assert np.array_equal(got, exp)
        assert (got[:50_000] == (1 << nf) - 1).all()


@pytest.mark.parametrize("n,filter_keys,fpr,slice20,sweeps", [
    (24_000_000, 200_000_000, 0.01, False, 1),   # 1825 2^20-bit slices -> one sweep of 2^21-bit bins
    (20_000_000, 10**9, 0.01, False, 2),         # C5's filter: 2 sweeps of 2^21-bit bins
    (20_000_000, 10**9, 0.01, True, 4),          # the same with 2^20-bit bins pinned: 4 sweeps
    (20_000_000, 200_000_000, 0.01, True, 2),    # a Walk32 filter (< 2^31 bits) in 2 sweeps of 2^20-bit bins
    (6_000_000, 10**9, 0.001, False, 4),         # k = 10: generic-k kernels keep 2^20-bit bins
])
def test_build_multi_sweep_steady_state(ctx, oracle, monkeypatch, n, filter_keys, fpr, slice20, sweeps):
    # partitioned builds of filters above 1024 bins: both bin widths, every word
    if slice20:
        monkeypatch.setenv("LSMB_SLICE_LOG2", "20")
    keys = keygen.key16(0x5EED0001, 0, n)
    nb, k = lsmbloom.params(filter_keys, fpr)
    assert lsmbloom.build_strategy(nb, n, k) == "partition"
    assert lsmbloom.build_sweeps(nb, n, k) == sweeps
    _cmp(ctx.build_fixed(keys, 16, nb, k), oracle.build_fixed_mt(keys, 16, nb, k, 16))


@pytest.mark.parametrize("n,filter_keys", [(150_000, 150_000), (1_000_000, 1_000_000), (3_500_000, 3_500_000),
                                           (50_000, 2_000_000)])
def test_build_tiled_mid_size_filters(ctx, oracle, n, filter_keys):
    # 160 KiB .. 4 MiB filters (compaction-sized SSTables): per-slice LDS tiles + OR-reduce
    keys = keygen.key16(0x7117ED, 0, n)
    nb, k = lsmbloom.params(filter_keys, 0.01)
    assert lsmbloom.build_strategy(nb, n) == "tiled"
    w = np.zeros(lsmbloom.num_words(nb), dtype=np.uint64)
    w[::97] = 0x8000000000000001  # OR-accumulate into existing bits
    ref = oracle.build_fixed(keys, 16, nb, k, words=w.copy())
    _cmp(ctx.build_fixed(keys, 16, nb, k, words=w), ref)


def test_build_tiled_varlen(ctx, oracle):
    data, offs = keygen.varlen(400_000)
    nb, k = lsmbloom.params(400_000, 0.01)
    assert lsmbloom.build_strategy(nb, 400_000) == "tiled"
    _cmp(ctx.build_var(data, offs, nb, k), oracle.build_var(data, offs, nb, k))


def test_build_few_keys_huge_filter_atomic(ctx, oracle):
    nb, k = lsmbloom.params(10**8, 0.01)
    keys = keygen.key16(0x1234, 0, 1000)
    assert lsmbloom.build_strategy(nb, 1000) == "atomic"
    _cmp(ctx.build_fixed(keys, 16, nb, k), oracle.build_fixed(keys, 16, nb, k))


def test_build_duplicate_heavy_overflow(ctx, oracle):
    # 2M copies of one key + 8M distinct: the 7 slices of the repeated key get
    # far more than their expected share, exercising the region-overflow path.
    n = 10_000_000
    keys = keygen.key16(0xD00D, 0, n)
    keys[: 2_000_000] = keys[0]
    nb, k = lsmbloom.params(n, 0.01)
    assert lsmbloom.build_strategy(nb, n) == "partition"
    _cmp(ctx.build_fixed(keys, 16, nb, k), oracle.build_fixed_mt(keys, 16, nb, k, 16))


def test_build_or_accumulates(ctx, oracle):
    n = 500_000
    nb, k = lsmbloom.params(2 * n, 0.01)
    a = keygen.key16(1, 0, n)
    b = keygen.key16(2, 0, n)
    w = ctx.build_fixed(a, 16, nb, k)
    w = ctx.build_fixed(b, 16, nb, k, words=w)
    ref = oracle.build_fixed(b, 16, nb, k, words=oracle.build_fixed(a, 16, nb, k))
    _cmp(w, ref)


@pytest.mark.parametrize("key_len", [1, 3, 4, 7, 8, 9, 12, 15, 16, 17, 31, 64, 100, 128, 129, 200,
                                     240, 241, 256, 300, 1024, 1025, 4000])
def test_build_fixed_len_vs_oracle(ctx, oracle, key_len):
    n = 20_000 if key_len <= 300 else 2000
    data = keygen.stream_bytes(0xABC + key_len, n * key_len)
    for fpr in (0.01,):
        nb, k = lsmbloom.params(n, fpr)
        _cmp(ctx.build_fixed(data, key_len, nb, k), oracle.build_fixed(data, key_len, nb, k))
    nb, k = lsmbloom.params(50 * n, 0.01)  # partition strategy for bigger filters
    _cmp(ctx.build_fixed(data, key_len, nb, k), oracle.build_fixed(data, key_len, nb, k))


def test_build_var_every_length_class(ctx, oracle):
    rng = np.random.default_rng(3)
    lens = list(range(0, 301)) * 20 + [511, 1023, 1024, 1025, 2048, 4097, 10000]
    rng.shuffle(lens)
    blob = keygen.stream_bytes(0x77, int(sum(lens)))
    offs = np.zeros(len(lens) + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    for n_exp in (len(lens), 40 * len(lens)):
        nb, k = lsmbloom.params(n_exp, 0.01)
        _cmp(ctx.build_var(blob, offs, nb, k), oracle.build_var(blob, offs, nb, k))


@pytest.mark.parametrize("tail", [1, 40, 64])
def test_build_var_partial_last_block(ctx, oracle, tail):
    """A last k_hash_var block of <= 64 keys that hold more than 1 KiB: the
    block's waves 1-3 have no key but still issue window pieces (LDS-DMA),
    which wave 0's lanes then read.  256 k + tail keys, the tail
    keys 200-256 B long, partition build (the k_hash_var path) vs the oracle."""
    rng = np.random.default_rng(0x7A11 + tail)
    n = 256 * 1000 + tail
    lens = rng.integers(8, 257, size=n).astype(np.uint64)
    lens[-tail:] = rng.integers(200, 257, size=tail)
    assert int(lens[-tail:].sum()) > 1024 or tail == 1
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = keygen.stream_bytes(0x7A11 + tail, int(offs[-1]))
    nb, k = lsmbloom.params(10_000_000, 0.01)
    assert lsmbloom.build_strategy(nb, n, k) == "partition"
    _cmp(ctx.build_var(blob, offs, nb, k), oracle.build_var(blob, offs, nb, k))


def test_build_walk_records_saturated_filter(ctx, oracle):
    """Var-len and odd-length keys into the saturated 2^32-1-bit filter
    (new(1e9, 0.01)): the hash kernels write walk records whose remainders
    are folds there (2^32 = 1 mod d), replayed by the 64-bit record walk in
    two sweeps; every word vs the oracle."""
    n = 3_000_000
    nb, k = lsmbloom.params(10**9, 0.01)
    assert nb == 2**32 - 1
    data, offs = keygen.varlen(n)
    assert lsmbloom.build_strategy(nb, n, k) == "partition" and lsmbloom.build_sweeps(nb, n, k) == 2
    _cmp(ctx.build_var(data, offs, nb, k), oracle.build_var_mt(data, offs, nb, k, 16))
    keys7 = np.ascontiguousarray(keygen.key16(0x5A7, 0, n)[:, :7])
    _cmp(ctx.build_fixed(keys7, 7, nb, k), oracle.build_fixed_mt(keys7, 7, nb, k, 16))


def test_build_var_c4_shape(ctx, oracle):
    n = 1_000_000
    data, offs = keygen.varlen(n)
    nb, k = lsmbloom.params(n, 0.01)
    _cmp(ctx.build_var(data, offs, nb, k), oracle.build_var(data, offs, nb, k))


def test_build_var_c4_10m_exact(ctx, oracle):
    """C4's key shape (8-256 B, tests/keygen.varlen) at 10 M keys into the
    C4 filter new(1e8, 0.01): the device build (HBM-resident keys, the bench's
    path) word-for-word against the multithreaded oracle."""
    import torch
    n = 10_000_000
    dev = torch.device("cuda:0")
    data_d, offs_d = ctx.gen_varlen_dev(n)
    data, offs = data_d.cpu().numpy(), offs_d.cpu().numpy().view(np.uint64)
    h_data, h_offs = keygen.varlen(1000)
    assert np.array_equal(offs[:1001], h_offs) and np.array_equal(data[:int(h_offs[-1])], h_data)
    nb, k = lsmbloom.params(100_000_000, 0.01)
    words = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    ctx.build_var_dev(data_d, offs_d, n, nb, k, words)
    ref = oracle.build_var_mt(data, offs, nb, k, 16)
    assert np.array_equal(words.cpu().numpy().view(np.uint64), ref)


def test_build_var_offsets_past_4gib(ctx, oracle):
    """Key data past 2 and 4 GiB with more blocks than k_hash_var's resident
    workgroups: 2 100 keys of 1 MiB, 300 k C4-shaped keys (offsets in
    [2^31, 2^32): the offsets' low dwords have bit 31 set), 2 100 more 1 MiB
    keys, 100 k C4-shaped keys (offsets above 2^32).  The 1 MiB keys are
    longer than the LDS window, so each is hashed from global memory by its
    lane.  ~1 580 blocks of 256 keys: more than 4 workgroups x 256 CUs, so
    blocks past the first 1 024 are reached through a workgroup's block loop
    in a grid-capped launch.  Partition build into new(1e8, 0.01) vs the oracle."""
    import torch
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0x4617)
    mib = lambda c: np.full(c, 1 << 20, np.uint64)
    small = lambda c: rng.integers(8, 257, size=c).astype(np.uint64)
    lens = np.concatenate([mib(2100), small(300_000), mib(2100), small(100_000)])
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    total = int(offs[-1])
    assert 2**31 < int(offs[2100]) < int(offs[302_100]) < 2**32 < int(offs[304_200])
    data_d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    offs_d = torch.from_numpy(offs.view(np.int64)).to(dev)
    n = lens.size
    nb, k = lsmbloom.params(100_000_000, 0.01)
    words = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    ctx.build_var_dev(data_d, offs_d, n, nb, k, words)
    got = words.cpu().numpy().view(np.uint64)
    data = data_d.cpu().numpy()
    del data_d
    ref = oracle.build_var_mt(data, offs, nb, k, 16)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("k", [1, 2, 7, 8, 9, 16, 17, 32, 33, 40])
def test_build_any_k(ctx, oracle, k):
    n = 200_000
    keys = keygen.key16(0xBEE + k, 0, n)
    for nb in (5000, 4_000_003):
        _cmp(ctx.build_fixed(keys, 16, nb, k), oracle.build_fixed(keys, 16, nb, k))


# ---------------------------------------------------------------- probe
def _c3_filters(oracle, nfilt=8, members=1000):
    nb, k = lsmbloom.params(members, 0.01)  # SSTableBuilder::new sizing at 1000
    fl, mem = [], []
    for f in range(nfilt):
        keys = keygen.key16(0xF000 + f, 0, members)
        fl.append((oracle.build_fixed(keys, 16, nb, k), nb, k))
        mem.append(keys)
    return fl, np.concatenate(mem)


@pytest.mark.parametrize("nfilt", [1, 3, 5, 7, 8, 9, 16, 17, 32])
def test_probe_sliced_vs_oracle(ctx, oracle, nfilt):
    fl, mem = _c3_filters(oracle, nfilt)
    q = 200_000
    rng = np.random.default_rng(nfilt)
    fresh = keygen.key16(0xAAAA, 0, q // 2)
    hits = mem[rng.integers(0, mem.shape[0], q - q // 2)]
    keys = np.concatenate([fresh, hits])
    got = ctx.probe(fl, keys, key_len=16)
    ref = oracle.probe(fl, keys, key_len=16)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("q,members", [(1, 1000), (63, 1000), (1025, 1000), (262_149, 1000), (786_532, 1000),
                                       (1_048_577, 1000), (1_310_720, 1000), (1_048_577, 5000)])
def test_probe_sliced_round_counts(ctx, oracle, q, members):
    """The C3 kernel walks the keys in grid-wide rounds (256 CUs x 1024 lanes
    on an MI355X), three in flight: one to five rounds, partial last rounds,
    and a batch smaller than one workgroup; new(5000, .01) filters (47 836
    bits, above Walk14's 2^14) take the same loop with the 32-bit walk."""
    fl, mem = _c3_filters(oracle, 8, members)
    rng = np.random.default_rng(q)
    keys = np.concatenate([keygen.key16(0xABCD, 0, q - q // 2), mem[rng.integers(0, mem.shape[0], q // 2)]])
    assert np.array_equal(ctx.probe(fl, keys, key_len=16), oracle.probe(fl, keys, key_len=16))


def test_probe_generic_mixed_filters(ctx, oracle):
    fl = []
    for i, (n, fpr) in enumerate([(1000, 0.01), (50_000, 0.001), (300_000, 0.05), (10, 0.5), (2_000_000, 0.01)]):
        nb, k = lsmbloom.params(n, fpr)
        keys = keygen.key16(0x5000 + i, 0, n)
        fl.append((oracle.build_fixed(keys, 16, nb, k), nb, k))
    fl.append((np.zeros(0, np.uint64), 0, 0))  # num_bits = 0, k = 0: always true
    q = 100_000
    keys = np.concatenate([keygen.key16(0x5001, 0, q // 2), keygen.key16(0x9999, 0, q // 2)])
    assert np.array_equal(ctx.probe(fl, keys, key_len=16), oracle.probe(fl, keys, key_len=16))
    data, offs = keygen.varlen(30_000)
    assert np.array_equal(ctx.probe(fl, data, offs), oracle.probe(fl, data, offs))


def test_probe_many_filters_64(ctx, oracle):
    fl = []
    for f in range(64):
        nb, k = lsmbloom.params(200 + 10 * f, 0.01)
        fl.append((oracle.build_fixed(keygen.key16(0x6000 + f, 0, 200), 16, nb, k), nb, k))
    keys = np.concatenate([keygen.key16(0x6000 + f, 0, 50) for f in range(64)] + [keygen.key16(1, 0, 5000)])
    assert np.array_equal(ctx.probe(fl, keys, key_len=16), oracle.probe(fl, keys, key_len=16))


def test_probe_varlen_keys_sliced(ctx, oracle):
    fl, _ = _c3_filters(oracle, 8)
    data, offs = keygen.varlen(100_000)
    assert np.array_equal(ctx.probe(fl, data, offs), oracle.probe(fl, data, offs))


# ---------------------------------------------------------------- device-resident API
def test_device_api_torch(ctx, oracle):
    import torch
    dev = torch.device("cuda:0")
    n = 1_000_003
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    torch.cuda.synchronize()
    host = keygen.key16(0x5EED0001, 0, n)
    assert np.array_equal(keys.cpu().numpy(), host)
    nb, k = lsmbloom.params(n, 0.01)
    words = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    ctx.build_fixed_dev(keys, 16, n, nb, k, words)
    torch.cuda.synchronize()
    ref = oracle.build_fixed(host, 16, nb, k)
    _cmp(words.cpu().numpy().view(np.uint64), ref)
    # unaligned base pointer -> generic fixed-length path
    raw = torch.zeros(n * 16 + 16, dtype=torch.uint8, device=dev)
    raw[3:3 + n * 16] = keys.reshape(-1)
    w2 = torch.zeros_like(words)
    ctx.build_fixed_dev(raw[3:], 16, n, nb, k, w2)
    torch.cuda.synchronize()
    assert torch.equal(words, w2)
    out = torch.zeros(n, dtype=torch.uint8, device=dev)
    ctx.probe_dev([(words, nb, k)], keys, n, out, key_len=16)
    torch.cuda.synchronize()
    assert bool(out.bool().all())


def test_or_reduce_dev(ctx):
    import torch
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    src = torch.randint(-2**62, 2**62, (4, 100_001), generator=g, dtype=torch.int64)
    dst = torch.randint(-2**62, 2**62, (100_001,), generator=g, dtype=torch.int64)
    ref = dst.clone()
    for j in range(4):
        ref |= src[j]
    d_dst, d_src = dst.to(dev), src.to(dev)
    ctx.or_reduce_dev(d_dst, d_src, 100_001, 4, 100_001)
    torch.cuda.synchronize()
    assert torch.equal(d_dst.cpu(), ref)


@pytest.mark.slow
def test_c2_full_size_bit_exact(ctx, oracle):
    """BASELINE C2 at full size: 100 M key16 into new(1e8, 0.01), every word."""
    import torch
    n = 100_000_000
    nb, k = lsmbloom.params(n, 0.01)
    assert (nb, k) == (956_715_292, 7)
    dev = torch.device("cuda:0")
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    words = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    ctx.build_fixed_dev(keys, 16, n, nb, k, words)
    torch.cuda.synchronize()
    got = words.cpu().numpy().view(np.uint64)
    del keys
    host = oracle.key16(0x5EED0001, 0, n)
    ref = oracle.build_fixed_mt(host, 16, nb, k, 16)
    _cmp(got, ref)
    assert_full_fixture(got, "c2")


def test_c2_exact10_full_size_fixture(ctx):
    """C2's exact 10 bits/key variant (num_bits = 1e9, k = 7):
    100 M key16 on the device, every word against the oracle's digest."""
    import torch
    n = 100_000_000
    dev = torch.device("cuda:0")
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    words = torch.zeros(lsmbloom.num_words(10 * n), dtype=torch.int64, device=dev)
    ctx.build_fixed_dev(keys, 16, n, 10 * n, 7, words)
    torch.cuda.synchronize()
    assert_full_fixture(words.cpu().numpy().view(np.uint64), "c2_exact10")


@pytest.mark.parametrize("fresh", [True, False])
def test_c5_shard0_fixture(ctx, fresh):
    """configs[4]'s per-GPU build: the first 125 M C5 keys (shard 0 of 8) into
    new(1e9, 0.01) = 2^32-1 bits (two sweeps of 2^21-bit bins), fresh and
    OR-accumulate into zeros, every word against the oracle's digest."""
    import torch
    n = 125_000_000
    nb, k = lsmbloom.params(1_000_000_000, 0.01)
    dev = torch.device("cuda:0")
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    if fresh:
        words = torch.full((lsmbloom.num_words(nb),), -1, dtype=torch.int64, device=dev)  # garbage: output-only
        ctx.build_fixed_dev_new(keys, 16, n, nb, k, words)
    else:
        words = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
        ctx.build_fixed_dev(keys, 16, n, nb, k, words)
    torch.cuda.synchronize()
    del keys
    assert_full_fixture(words.cpu().numpy().view(np.uint64), "c5_shard0")


def test_c5_full_size_shards_or_equal_monolithic(ctx):
    """C5 data path at full size on one GPU: 1e9 16-B keys, filter new(1e9, 0.01)
    (2^32-1 bits, 512 MiB).  Eight shard builds (one per would-be rank) merged
    with the native OR-reduce must equal the monolithic build of all 1e9 keys
    (OR is associative, commutative and idempotent), every sampled member must
    probe positive, and the fill ratio must match 1 - exp(-kN/m).  These are
    size-independent properties, and the monolithic filter's digest equals
    the oracle's full-size C5 filter (tests/golden/fullsize_fixture.json)."""
    import math

    import torch
    dev = torch.device("cuda:0")
    N, G = 1_000_000_000, 8
    nb, k = lsmbloom.params(N, 0.01)
    assert nb == 2**32 - 1
    nw = lsmbloom.num_words(nb)
    keys = torch.empty((N, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, N, keys)
    mono = torch.zeros(nw, dtype=torch.int64, device=dev)
    ctx.build_fixed_dev(keys, 16, N, nb, k, mono)
    parts = torch.zeros((G, nw), dtype=torch.int64, device=dev)
    per = N // G
    for g in range(G):
        ctx.build_fixed_dev(keys[g * per:(g + 1) * per], 16, per, nb, k, parts[g])
    merged = torch.zeros(nw, dtype=torch.int64, device=dev)
    ctx.or_reduce_dev(merged, parts, nw, G, nw)
    ctx.sync()
    torch.cuda.synchronize()
    assert torch.equal(merged, mono)
    del parts, merged
    host_words = mono.cpu().numpy().view(np.uint64)
    assert_full_fixture(host_words, "c5")  # every word == the oracle's C5 filter
    ones = int(np.unpackbits(host_words.view(np.uint8)).sum())
    assert abs(ones / nb - (1 - math.exp(-k * N / nb))) < 1e-3, ones / nb
    sample = keys[::1_000_003][:1000].contiguous()
    hs = sample.cpu().numpy()
    f = BloomFilter(host_words, k, nb)
    assert all(f.may_contain(bytes(hs[i])) for i in range(0, hs.shape[0], 50))  # host single-key path
    out = torch.zeros(sample.shape[0], dtype=torch.uint8, device=dev)
    ctx.probe_dev([(mono, nb, k)], sample, sample.shape[0], out, key_len=16)
    torch.cuda.synchronize()
    assert bool(out.bool().all()), int(out.sum().item())
    del keys, mono
    torch.cuda.empty_cache()


def test_c4_full_size_properties(ctx, oracle):
    """C4 at full size: 1e8 var-len keys (8-256 B, ~13.2 GB) on the device.
    The monolithic build equals the OR of four shard builds (each shard's
    offsets rebased to its own data slice), sampled members probe positive
    (and agree with the host single-key path), and the fill ratio is analytic.
    The word-exact oracle comparison of this path at 10 M keys is
    test_build_var_c4_10m_exact."""
    import math

    import torch
    import sys
    import time
    t0 = time.time()

    def tick(what):
        print("[c4 %.1fs] %s" % (time.time() - t0, what), file=sys.stderr, flush=True)
    N, G = 100_000_000, 4
    data, offs = ctx.gen_varlen_dev(N)
    tick("generated")
    nb, k = lsmbloom.params(N, 0.01)
    nw = lsmbloom.num_words(nb)
    dev = data.device
    mono = torch.zeros(nw, dtype=torch.int64, device=dev)
    ctx.build_var_dev(data, offs, N, nb, k, mono)
    torch.cuda.synchronize()
    tick("monolithic build")
    merged = torch.zeros(nw, dtype=torch.int64, device=dev)
    per = N // G
    for g in range(G):
        o0, o1 = int(offs[g * per].item()), int(offs[(g + 1) * per].item())
        so = (offs[g * per:(g + 1) * per + 1] - o0).contiguous()
        part = torch.zeros(nw, dtype=torch.int64, device=dev)
        ctx.build_var_dev(data[o0:o1], so, per, nb, k, part)
        merged |= part
        del part, so
    ctx.sync()
    torch.cuda.synchronize()
    tick("shard builds")
    assert torch.equal(merged, mono)
    del merged
    host_words = mono.cpu().numpy().view(np.uint64)
    assert_full_fixture(host_words, "c4")  # every word == the oracle's C4 filter
    ones = int(np.bitwise_count(host_words).sum(dtype=np.uint64))
    tick("fill counted")
    assert abs(ones / nb - (1 - math.exp(-k * N / nb))) < 1e-3, ones / nb
    idx = list(range(0, N, 997_331))[:100]
    f = BloomFilter(host_words, k, nb)
    oh = offs.cpu().numpy()
    tick("offsets to host")
    for i in idx:
        key = bytes(data[int(oh[i]):int(oh[i + 1])].cpu().numpy())
        assert f.may_contain(key)
    del data, offs, mono
    torch.cuda.empty_cache()


# ---------------------------------------------------------------- C3 at full size
def test_c3_full_size_every_answer(ctx, oracle):
    """C3 (10 M lookups x 8 SST filters, configs[2]) with
    every answer byte compared, not a sample: the plain batched probe
    (may_contain per table, src/sstable/reader.rs:197) and the filter-set form
    with SSTable::get's range pre-check (reader.rs:192-199, shape of
    tests/bloom_sstable_integration_tests.rs:66-113), same-size and mixed-size
    tables, against the oracle (tests/c3_ref.py: bench.py's workload)."""
    import torch
    import c3_ref
    Q, F = 10_000_000, 8
    mask, fset_ref, mixed_ref = c3_ref.answers(oracle, Q, F, threads=16)
    members, q_host, _ = c3_ref.workload(oracle, Q, F)
    dev = torch.device("cuda:0")
    nb, k = lsmbloom.params(1000, 0.01)
    mem = torch.from_numpy(members).to(dev)
    filt = []
    for f in range(F):
        w = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
        ctx.build_fixed_dev(mem[f * 1000:(f + 1) * 1000], 16, 1000, nb, k, w)
        filt.append((w, nb, k))
    q = torch.from_numpy(q_host).to(dev)
    out = torch.zeros((Q, 1), dtype=torch.uint8, device=dev)
    ctx.probe_dev(filt, q, Q, out, key_len=16)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    bad = np.flatnonzero(got[:, 0] != mask[:, 0])
    assert bad.size == 0, "probe answers differ at %d rows, first %s" % (bad.size, bad[:5])
    fout = torch.zeros(Q, dtype=torch.int64, device=dev)
    for mixed in (False, True):
        fs = lsmbloom.FilterSet(ctx)
        nb4, k4 = lsmbloom.params(4000, 0.01)
        for f in range(F):
            if mixed and f >= F // 2:
                rows = oracle.key16(0xF100 + f, 0, 4000)
                bf = lsmbloom.BloomFilter(oracle.build_fixed(rows, 16, nb4, k4), k4, nb4)
            else:
                rows = members[f * 1000:(f + 1) * 1000]
                bf = lsmbloom.BloomFilter(filt[f][0].cpu().numpy().view(np.uint64), k, nb)
            lo, hi = c3_ref.sorted_bounds(rows)
            assert fs.add_filter(bf, lo.tobytes(), hi.tobytes()) == f
        fs.probe_dev(q, Q, fout, key_len=16)
        torch.cuda.synchronize()
        ref = mixed_ref if mixed else fset_ref
        g = fout.cpu().numpy().view(np.uint64)
        bad = np.flatnonzero(g != ref)
        assert bad.size == 0, "filter-set (mixed=%s) answers differ at %d rows" % (mixed, bad.size)
        fs.close()
