"""CRC-32 of bloom blocks (the optional checksum over the
words; the reference's bloom block has none).  The CRC is crc32fast::hash's
(IEEE, the store's WAL/manifest checksum, src/wal/record.rs:96,122), which is
zlib.crc32: Python's zlib is the checker here."""
import os
import zlib

import numpy as np
import pytest

import keygen
import lsmbloom


def test_host_crc32_matches_zlib():
    rng = np.random.default_rng(5)
    for n in [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 63, 64, 65, 511, 512, 513, 4096, 100_003]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert lsmbloom.crc32(b) == zlib.crc32(b), n
        assert lsmbloom.crc32(b, 0x12345678) == zlib.crc32(b, 0x12345678), n


def test_crc32_combine():
    a, b = os.urandom(1234), os.urandom(98765)
    assert lsmbloom.crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)
    assert lsmbloom.crc32_combine(zlib.crc32(a), zlib.crc32(b""), 0) == zlib.crc32(a)
    assert lsmbloom.crc32_combine(0, zlib.crc32(b), len(b)) == zlib.crc32(b)


def test_build_block_crc_host_path():
    # at most lsmb_host_max_keys() keys: the library's host loop, no context
    keys = keygen.key16(0x5EED0001, 0, 1000)
    nb, k = lsmbloom.params(1000, 0.01)
    ctx = lsmbloom.Context.__new__(lsmbloom.Context)
    ctx.h = None
    block, crc = ctx.build_block_crc(keys, nb, k, key_len=16)
    assert crc == zlib.crc32(block.tobytes())


@pytest.mark.gpu
def test_crc32_dev_lengths_and_alignment():
    # offsets 4, 8, 12: 4-B aligned (dword loads); 0, 16: 16-B loads; odd: byte loop
    import torch
    ctx = lsmbloom.Context(0)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, (3 << 20) + 77, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    kb = 128 * 1024
    for off, n in [(0, 0), (0, 1), (0, 511), (0, 512), (0, 513), (0, kb - 1), (0, kb), (0, kb + 1),
                   (0, 3 * kb + 4099), (1, 1000), (3, kb + 5), (4, 2 * kb), (8, kb + 7), (12, 3 * kb + 1),
                   (16, kb), (0, host.size), (5, host.size - 5)]:
        got = ctx.crc32_dev(d[off:off + n], n)
        assert got == zlib.crc32(host[off:off + n].tobytes()), (off, n)
    # appended to a prefix CRC
    pre = zlib.crc32(b"header bytes")
    assert ctx.crc32_dev(d[:kb + 9], kb + 9, crc=pre) == zlib.crc32(host[:kb + 9].tobytes(), pre)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,filter_n", [(2_000_000, 2_000_000), (3000, 3000), (100_000_000, 100_000_000)])
def test_build_block_crc_device(n, filter_n):
    # device builds: the words' CRC is computed on the device copy
    import torch
    ctx = lsmbloom.Context(0)
    nb, k = lsmbloom.params(filter_n, 0.01)
    if n == 100_000_000:  # C2 at full size, keys from the device generator
        keys = torch.empty((n, 16), dtype=torch.uint8, device="cuda:0")
        ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
        keys = keys.cpu().numpy()
    else:
        keys = keygen.key16(0x5EED0001, 0, n)
    block, crc = ctx.build_block_crc(keys, nb, k, key_len=16)
    assert crc == zlib.crc32(block.tobytes())
    assert np.array_equal(block, ctx.build_block(keys, nb, k, key_len=16))
    ctx.close()


@pytest.mark.gpu
def test_fset_add_checked(oracle):
    ctx = lsmbloom.Context(0)
    fs = lsmbloom.FilterSet(ctx)
    keys = keygen.key16(0x5EED0900, 0, 5000)
    nb, k = lsmbloom.params(5000, 0.01)
    block = oracle.serialize(oracle.build_fixed(keys, 16, nb, k), nb, k)
    rows = sorted(bytes(r) for r in keys)
    good = zlib.crc32(bytes(block))
    with pytest.raises(lsmbloom.Corruption):
        fs.add_checked(block, good ^ 1, rows[0], rows[-1])
    assert fs.live_mask() == 0
    s = fs.add_checked(block, good, rows[0], rows[-1])
    assert fs.live_mask() == 1 << s
    assert all(int(x) >> s & 1 for x in fs.probe(keys[:1000], key_len=16))
    fs.close()
    ctx.close()
