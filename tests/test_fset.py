"""Device-resident filter sets (lsmb_fset): the batched form of the two checks
SSTable::get makes before reading the index (src/sstable/reader.rs:192-199):

    min_key <= key <= max_key  (Rust [u8] Ord: byte-wise, a proper prefix first)
    && bloom.may_contain(key)

Expected answers come from the CPU oracle's may_contain (the checker) and
Python's bytes ordering, which is the same lexicographic order as Rust's.
"""
import ctypes

import numpy as np
import pytest

import keygen
import lsmbloom
from lsmbloom import BloomFilter, FilterSet


def expected_masks(oracle, tables, keys):
    """tables: {slot: (words, num_bits, k, lo, hi)} -> list of uint64 masks."""
    data, offs = keygen.pack(keys)
    out = [0] * len(keys)
    for s, (w, nb, k, lo, hi) in tables.items():
        hit = oracle.probe([(w, nb, k)], data, offsets=offs)[:, 0]
        for i, key in enumerate(keys):
            if hit[i] and lo <= key <= hi:
                out[i] |= 1 << s
    return out


def sst_tables(oracle, ntab, per, seed):
    """ntab SSTable-like runs of `per` sorted keys each (L0-style overlapping
    ranges for even tables, disjoint for odd ones), filters sized as
    SSTableBuilder::with_estimated_keys(per) does (src/sstable/builder.rs:74)."""
    rng = np.random.default_rng(seed)
    tabs = []
    for t in range(ntab):
        base = t * 10_000 if t % 2 else (t // 2) * 3_000
        ids = np.sort(rng.choice(20_000, size=per, replace=False)) + base
        keys = [b"user%08d" % i for i in ids]
        nb, k = lsmbloom.params(per, 0.01)
        data, offs = keygen.pack(keys)
        w = oracle.build_var(data, offs, nb, k)
        tabs.append((keys, w, nb, k))
    return tabs


def test_fset_open_without_context_is_einval():
    h = ctypes.c_void_p()
    assert lsmbloom.lib().lsmb_fset_open(None, ctypes.byref(h)) == lsmbloom.LSMB_EINVAL
    assert lsmbloom.lib().lsmb_fset_live_mask(None) == 0


@pytest.mark.gpu
def test_fset_matches_range_and_bloom_checks(oracle):
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    tabs = sst_tables(oracle, 12, 1000, 7)
    tables = {}
    for keys, w, nb, k in tabs:
        s = fs.add(oracle.serialize(w, nb, k), keys[0], keys[-1])
        tables[s] = (w, nb, k, keys[0], keys[-1])
    assert fs.live_mask() == (1 << len(tabs)) - 1
    rng = np.random.default_rng(11)
    q = [kk for keys, _, _, _ in tabs for kk in keys[::7]]                     # members
    q += [b"user%08d" % i for i in rng.integers(0, 140_000, 20_000)]          # mostly absent
    q += [keys[0] for keys, *_ in tabs] + [keys[-1] for keys, *_ in tabs]     # inclusive bounds
    q += [b"", b"user", b"user0", b"user00000000\x00", b"zzz", b"\xff" * 40]  # prefixes, extremes
    q += [keys[0][:-1] for keys, *_ in tabs] + [keys[-1] + b"\x00" for keys, *_ in tabs]
    got = fs.probe_keys(q)
    exp = expected_masks(oracle, tables, q)
    assert [int(x) for x in got] == exp
    # every member is reported by its own table
    for s, (keys, *_rest) in enumerate(tabs):
        m = fs.probe_keys(keys)
        assert all(int(x) >> s & 1 for x in m)
    fs.close()
    ctx.close()


@pytest.mark.gpu
def test_fset_fixed_len_keys_and_device_probe(oracle):
    import torch

    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    tables = {}
    for t in range(8):
        keys = keygen.key16(0x5EED0100 + t, 0, 5000)
        rows = sorted(bytes(r) for r in keys)
        nb, k = lsmbloom.params(5000, 0.01)
        w = oracle.build_fixed(keys, 16, nb, k)
        s = fs.add_filter(BloomFilter(w, k, nb), rows[len(rows) // 4], rows[3 * len(rows) // 4])
        tables[s] = (w, nb, k, rows[len(rows) // 4], rows[3 * len(rows) // 4])
    q = np.concatenate([keygen.key16(0x5EED0100 + t, 0, 3000) for t in range(8)]
                       + [keygen.key16(0x5EED0200, 0, 20_000)])
    got = fs.probe(q, key_len=16)
    exp = expected_masks(oracle, tables, [bytes(r) for r in q])
    assert [int(x) for x in got] == exp
    dq = torch.from_numpy(np.ascontiguousarray(q)).to("cuda:0")
    dout = torch.zeros(q.shape[0], dtype=torch.int64, device="cuda:0")
    fs.probe_dev(dq, q.shape[0], dout, key_len=16)
    torch.cuda.synchronize()
    assert np.array_equal(dout.cpu().numpy().view(np.uint64), got)
    # probes on many streams (per-request / pooled streams): the set
    # tracks at most 4 and waits for the evicted one; adds and removes between
    # them still see every answer right
    streams = [torch.cuda.Stream("cuda:0") for _ in range(9)]
    outs = [torch.zeros_like(dout) for _ in streams]
    for rep in range(3):
        for st, o in zip(streams, outs):
            fs.probe_dev(dq, q.shape[0], o, key_len=16, stream=st.cuda_stream)
        extra = fs.add_filter(BloomFilter(tables[0][0], tables[0][2], tables[0][1]), b"", b"")  # empty-range table
        fs.remove(extra)
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint64), got)
    # unaligned fixed-length keys (FixedN path)
    q7 = np.ascontiguousarray(q[:5000, :7])
    got7 = fs.probe(q7, key_len=7)
    assert [int(x) for x in got7] == expected_masks(oracle, tables, [bytes(r) for r in q7])
    fs.close()
    ctx.close()


@pytest.mark.gpu
def test_fset_saturated_and_mixed_size_filters(oracle):
    # one 2^32-1-bit filter (new(1e9, .01)) next to SST-sized ones in one set
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    tables = {}
    for t, (n, sized) in enumerate([(200_000, 10**9), (5000, 5000), (1000, 1000)]):
        keys = keygen.key16(0x5EED0300 + t, 0, n)
        rows = sorted(bytes(r) for r in keys)
        nb, k = lsmbloom.params(sized, 0.01)
        w = oracle.build_fixed(keys, 16, nb, k)
        s = fs.add_filter(BloomFilter(w, k, nb), rows[0], rows[-1])
        tables[s] = (w, nb, k, rows[0], rows[-1])
    q = np.concatenate([keygen.key16(0x5EED0300 + t, 0, 1000) for t in range(3)]
                       + [keygen.key16(0x5EED0400, 0, 5000)])
    got = fs.probe(q, key_len=16)
    assert [int(x) for x in got] == expected_masks(oracle, tables, [bytes(r) for r in q])
    fs.close()
    ctx.close()


@pytest.mark.gpu
def test_fset_add_remove_reuse_and_limits(oracle):
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    assert fs.probe_keys([b"a", b"b"]).tolist() == [0, 0]  # empty set
    nb, k = lsmbloom.params(100, 0.01)
    slots = []
    for t in range(64):
        w = np.zeros(lsmbloom.num_words(nb), np.uint64)
        oracle.insert(w, nb, k, b"k%02d" % t)
        slots.append(fs.add_filter(BloomFilter(w, k, nb), b"k%02d" % t, b"k%02d" % t))
    assert slots == list(range(64))
    with pytest.raises(ValueError):
        fs.add_filter(BloomFilter(np.zeros(lsmbloom.num_words(nb), np.uint64), k, nb), b"", b"")
    m = fs.probe_keys([b"k%02d" % t for t in range(64)])
    assert [int(x) for x in m] == [1 << t for t in range(64)]
    fs.remove(5)
    fs.remove(40)
    with pytest.raises(ValueError):
        fs.remove(5)
    assert fs.live_mask() == ((1 << 64) - 1) & ~(1 << 5) & ~(1 << 40)
    assert int(fs.probe_keys([b"k05"])[0]) == 0
    w = np.zeros(lsmbloom.num_words(nb), np.uint64)
    oracle.insert(w, nb, k, b"new")
    assert fs.add(oracle.serialize(w, nb, k), b"a", b"z") == 5  # lowest free slot
    got = int(fs.probe_keys([b"new"])[0])
    assert got >> 5 & 1 and not got >> 40 & 1
    fs.close()
    ctx.close()


@pytest.mark.gpu
def test_fset_add_rejects_corrupt_blocks_like_deserialize(oracle):
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    nb, k = lsmbloom.params(100, 0.01)
    good = oracle.serialize(np.zeros(lsmbloom.num_words(nb), np.uint64), nb, k)
    for bad in (b"", b"\xff\xff\xff\xff", bytes([7, 0, 0, 0, 0xE8, 3, 0, 0, 100, 0, 0, 0]),
                good + b"extra", good[:-1]):
        with pytest.raises(lsmbloom.Corruption):
            fs.add(bad, b"a", b"z")
    assert fs.live_mask() == 0
    # num_bits == 0 with k > 0: the reference would panic (% by zero) on probe
    zero = bytes([7, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0])
    with pytest.raises(ValueError):
        fs.add(zero, b"a", b"z")
    # k == 0: may_contain is vacuously true, so only the range decides
    s = fs.add(bytes([0, 0, 0, 0]) + good[4:], b"b", b"c")
    assert [int(x) for x in fs.probe_keys([b"a", b"b", b"bz", b"c", b"c\x00"])] == [0, 1 << s, 1 << s, 1 << s, 0]
    fs.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ntab,n,fpr", [(5, 800, 0.05), (12, 800, 0.01), (20, 800, 0.01), (33, 800, 0.001),
                                        (40, 500, 0.01), (64, 500, 0.01)])
def test_fset_same_sized_sliced_table_widths(oracle, ntab, n, fpr):
    # every filter of the set shares (num_bits, k): the bit-sliced LDS table
    # path at 8/16/32/64-bit entries (after removing slot 1: 4, 11, 19 / 32,
    # 39 and 63 filters; each table within 64 KiB of LDS) and k != 7, with a
    # non-identity slot -> output-bit mapping (slot 1 is gone)
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    nb, k = lsmbloom.params(n, fpr)
    tables = {}
    for t in range(ntab):
        keys = keygen.key16(0x5EED0500 + t, 0, n)
        rows = sorted(bytes(r) for r in keys)
        w = oracle.build_fixed(keys, 16, nb, k)
        lo, hi = rows[t % 3 * 100], rows[-1 - t % 5 * 100]
        s = fs.add_filter(BloomFilter(w, k, nb), lo, hi)
        tables[s] = (w, nb, k, lo, hi)
    fs.remove(1)
    del tables[1]
    q = np.concatenate([keygen.key16(0x5EED0500 + t, 0, 300) for t in range(ntab)]
                       + [keygen.key16(0x5EED0600, 0, 3000)])
    got = fs.probe(q, key_len=16)
    assert [int(x) for x in got] == expected_masks(oracle, tables, [bytes(r) for r in q])
    fs.close()
    ctx.close()


@pytest.mark.gpu
def test_fset_bounds_sharing_16_byte_prefixes(oracle):
    # range checks first order by the zero-padded 16-byte prefixes; ties fall
    # to lengths (both <= 16 B) or the full byte compare
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    P = b"0123456789abcdef"
    nb, k = lsmbloom.params(64, 0.01)
    bounds = [(P, P + b"\x00"), (P + b"a", P + b"m"), (P[:15], P), (P[:8] + b"\x00" * 8, P[:8] + b"\x00" * 9),
              (b"", P[:3]), (P + b"zz" * 10, P + b"zz" * 10 + b"\x01")]
    q = [P, P[:15], P + b"\x00", P + b"\x00\x00", P + b"a", P + b"m", P + b"ma", P + b"b" * 30, P[:14],
         P[:8] + b"\x00" * 7, P[:8] + b"\x00" * 8, P[:8] + b"\x00" * 9, P[:8] + b"\x00" * 10, b"", P[:3],
         P[:3] + b"\x00", P + b"zz" * 10, P + b"zz" * 10 + b"\x00", P + b"zz" * 10 + b"\x01\x00", P[:8]]
    tables = {}
    for lo, hi in bounds:
        w = np.zeros(lsmbloom.num_words(nb), np.uint64)
        for key in q:
            oracle.insert(w, nb, k, key)  # every query a member: the range decides
        s = fs.add_filter(BloomFilter(w, k, nb), lo, hi)
        tables[s] = (w, nb, k, lo, hi)
    got = fs.probe_keys(q)
    assert [int(x) for x in got] == expected_masks(oracle, tables, q)
    fs.close()
    ctx.close()


def _in_range16(rows, lo, hi):
    """lo <= key <= hi for 16-byte keys (n x 16 uint8) in Rust [u8] order."""
    def cmp(bound):  # -1 / 0 / 1 per row: key vs bound
        b = np.frombuffer(bound[:16].ljust(16, b"\x00"), np.uint8)
        d = rows.astype(np.int16) - b.astype(np.int16)
        first = np.argmax(d != 0, axis=1)
        c = np.sign(d[np.arange(rows.shape[0]), first]).astype(np.int8)
        # equal first min(16, len) bytes: the shorter one orders first
        eqp = np.all(rows[:, :min(16, len(bound))] == b[:min(16, len(bound))], axis=1)
        c[eqp] = 0 if len(bound) == 16 else (1 if len(bound) < 16 else -1)
        return c
    return (cmp(lo) >= 0) & (cmp(hi) <= 0)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [70_001, 524_289, 1_310_731])
def test_fset_sliced_round_counts_and_long_bounds(oracle, q):
    """The C3-shaped filter-set kernel (16-B keys, new(1000, .01) tables) over
    several grid-strides and a partial last one; bounds longer than 16 bytes
    that share a key's first 16 take the full byte compare, which re-reads
    that key from memory."""
    import torch

    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    nb, k = lsmbloom.params(1000, 0.01)
    members = [keygen.key16(0x5EED0700 + t, 0, 1000) for t in range(8)]
    keys = np.concatenate([keygen.key16(0x5EED0800, 0, q - q // 2)]
                          + [members[t][np.random.default_rng(t).integers(0, 1000, q // 2 // 8 + 1)] for t in range(8)])[:q]
    k0, k1 = bytes(keys[5]), bytes(keys[q // 2 + 3])
    tables = {}
    for t in range(8):
        rows = sorted(bytes(r) for r in members[t])
        lo, hi = [(rows[0], rows[-1]), (k0 + b"\x00", b"\xff" * 20), (k0[:15], k0 + b"\x07"),
                  (b"", k1 + b"\x00\x01"), (k1, k1), (rows[100], rows[900]), (k0 + b"a" * 8, k1 + b"b" * 5),
                  (b"\x00" * 17, b"\xff" * 16)][t]
        w = oracle.build_fixed(members[t], 16, nb, k)
        s = fs.add_filter(BloomFilter(w, k, nb), lo, hi)
        tables[s] = (w, lo, hi)
    exp = np.zeros(q, np.uint64)
    for s, (w, lo, hi) in tables.items():
        hit = oracle.probe([(w, nb, k)], keys, key_len=16)[:, 0].astype(bool)
        exp |= (hit & _in_range16(keys, lo, hi)).astype(np.uint64) << np.uint64(s)
    dq = torch.from_numpy(np.ascontiguousarray(keys)).to("cuda:0")
    dout = torch.zeros(q, dtype=torch.int64, device="cuda:0")
    fs.probe_dev(dq, q, dout, key_len=16)
    torch.cuda.synchronize()
    assert np.array_equal(dout.cpu().numpy().view(np.uint64), exp)
    fs.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mixed", [False, True])
def test_fset_random_ranges_region_lookup(oracle, mixed):
    """The range pre-check as one rank search over the sorted distinct bounds:
    random ranges with shared bounds, empty ranges (min > max), single-key
    ranges, and queries equal to / between / outside the bounds, with var-len
    keys up to 40 bytes (16-byte prefix ties resolved by the full compare).
    Same-sized filters take the sliced kernel, mixed sizes the per-filter one."""
    rng = np.random.default_rng(11 + mixed)
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    alphabet = [b"", b"a", b"ab", b"0123456789abcdef", b"0123456789abcdef\x00", b"0123456789abcdefz",
                b"0123456789abcdefzz" * 2, b"b", b"zz", b"\xff" * 17]

    def rnd_key():
        base = alphabet[rng.integers(len(alphabet))]
        return base + bytes(rng.integers(0, 256, size=rng.integers(0, 4), dtype=np.uint8))

    q = [rnd_key() for _ in range(3000)]
    tables = {}
    for t in range(30):
        a, b = rnd_key(), rnd_key()
        if t % 7 == 0:
            b = a  # single-key range
        if t % 5 == 0 and a < b:
            a, b = b, a  # empty range: min > max holds no key
        if t % 4 == 1 and tables:
            a = list(tables.values())[0][3]  # a shared bound
        n = 100 if not mixed else [100, 5000, 20000][t % 3]
        nb, k = lsmbloom.params(n, 0.01)
        w = np.zeros(lsmbloom.num_words(nb), np.uint64)
        for key in q[t::7]:
            oracle.insert(w, nb, k, key)
        s = fs.add_filter(BloomFilter(w, k, nb), a, b)
        tables[s] = (w, nb, k, a, b)
    got = fs.probe_keys(q)
    assert [int(x) for x in got] == expected_masks(oracle, tables, q)
    for s in (3, 17):
        fs.remove(s)
        del tables[s]
    got = fs.probe_keys(q)
    assert [int(x) for x in got] == expected_masks(oracle, tables, q)
    fs.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [
    [1000] * 8 + [3000] * 8 + [500] * 2,          # three classes, all in LDS tables
    [100 * (i + 1) for i in range(11)],            # 11 classes: 8 in LDS, the rest walked
    [1000] * 40 + [2000] * 3,                      # 40-member class (64-bit entries) + a small one
    [1000, 200_000, 1000, 50_000, 300],            # classes too big for LDS next to small ones
])
def test_fset_mixed_size_classes(oracle, sizes):
    """Mixed-size sets: one bit-sliced LDS table per (num_bits, k) class
    (k_fset_classes), classes that do not fit walked from L2, output bits
    mapped back to slots (slot 2 removed: a non-identity mapping)."""
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    tables = {}
    q = []
    for t, n in enumerate(sizes):
        keys = keygen.key16(0x5EED0700 + t, 0, min(n, 2000))
        rows = sorted(bytes(r) for r in keys)
        nb, k = lsmbloom.params(n, 0.01)
        w = oracle.build_fixed(keys, 16, nb, k)
        lo, hi = rows[t % 4 * 50], rows[-1 - t % 3 * 50]
        s = fs.add_filter(BloomFilter(w, k, nb), lo, hi)
        tables[s] = (w, nb, k, lo, hi)
        q.append(keys[:300])
    # a k = 0 filter (may_contain vacuously true: only the range decides) is walked
    nb0 = lsmbloom.params(1000, 0.01)[0]
    w0 = np.zeros(lsmbloom.num_words(nb0), np.uint64)
    s0 = fs.add_filter(BloomFilter(w0, 0, nb0), b"\x00", b"\x80")
    tables[s0] = (w0, nb0, 0, b"\x00", b"\x80")
    fs.remove(2)
    del tables[2]
    q = np.concatenate(q + [keygen.key16(0x5EED0800, 0, 5000)])
    got = fs.probe(q, key_len=16)
    assert [int(x) for x in got] == expected_masks(oracle, tables, [bytes(r) for r in q])
    fs.close()
    ctx.close()


@pytest.mark.gpu
def test_fset_mixed_size_classes_varlen_keys(oracle):
    """Mixed-size classes probed with variable-length keys (k_fset_classes'
    VarLen instance: one workgroup per CU, unlike the 16-B-key instance), a
    class below 2^14 bits (Mod14 walk) next to bigger ones (Mod32 walk)."""
    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    data, offs = keygen.varlen(24_000)
    keys = [bytes(data[offs[i]:offs[i + 1]]) for i in range(24_000)]
    tables = {}
    for t, n in enumerate([1000, 4000, 1000, 4000, 30_000, 1000]):
        mem = keys[t * 3000:t * 3000 + min(n, 3000)]
        d, o = keygen.pack(mem)
        nb, k = lsmbloom.params(n, 0.01)
        w = oracle.build_var(d, o, nb, k)
        rows = sorted(mem)
        lo, hi = rows[t % 3 * 10], rows[-1 - t % 2 * 10]
        s = fs.add_filter(BloomFilter(w, k, nb), lo, hi)
        tables[s] = (w, nb, k, lo, hi)
    fs.remove(1)
    del tables[1]
    q = keys[:20_000:3] + keys[18_000:]
    d, o = keygen.pack(q)
    got = fs.probe(d, offsets=o)
    assert [int(x) for x in got] == expected_masks(oracle, tables, q)
    fs.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [(1000,) * 8, (1000, 4000) * 4, (1000,) * 5 + (10 ** 9,), (1000,) * 12])
def test_fset_compact_rows(oracle, sizes):
    """lsmb_fset_probe_dev_rows: answer rows of 1, 2 or 4 bytes are the u64
    rows' low bytes on every kernel path (same-size sliced table, size
    classes, the generic L2 walk next to a saturated filter), and a live slot
    that does not fit the row width is LSMB_EINVAL."""
    import torch

    ctx = lsmbloom.Context(0)
    fs = FilterSet(ctx)
    for t, m in enumerate(sizes):
        nk = min(m, 3000)
        keys = keygen.key16(0x5EED0400 + t, 0, nk)
        rows = sorted(bytes(r) for r in keys)
        nb, k = lsmbloom.params(m, 0.01)
        fs.add_filter(BloomFilter(oracle.build_fixed(keys, 16, nb, k), k, nb), rows[nk // 5], rows[4 * nk // 5])
    q = np.concatenate([keygen.key16(0x5EED0400 + t, 0, 2000) for t in range(len(sizes))]
                       + [keygen.key16(0x5EED0500, 0, 30_000)])
    n = q.shape[0]
    dq = torch.from_numpy(np.ascontiguousarray(q)).to("cuda:0")
    full = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    fs.probe_dev(dq, n, full, key_len=16)
    torch.cuda.synchronize()
    ref = full.cpu().numpy().view(np.uint64)
    assert ref.any()
    for rb, dt in ((1, np.uint8), (2, np.uint16), (4, np.uint32)):
        out = torch.full((n * rb,), 0xA5, dtype=torch.uint8, device="cuda:0")
        if len(sizes) > 8 * rb:
            with pytest.raises(ValueError, match="does not fit"):  # LSMB_EINVAL, as the mirror raises it
                fs.probe_dev(dq, n, out, key_len=16, row_bytes=rb)
            continue
        fs.probe_dev(dq, n, out, key_len=16, row_bytes=rb)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(dt)
        assert np.array_equal(got, ref.astype(dt)), rb
    fs.close()
    ctx.close()
