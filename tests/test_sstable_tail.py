"""SSTable bloom-block placement and tail codec, host side.

The bloom block here comes from the CPU oracle (test infrastructure); the GPU
build of the same block is in tests/test_gpu_block.py.  Mirrors the reference's
footer_has_bloom_block_info (tests/bloom_sstable_integration_tests.rs:142-174)
and the footer / meta codecs (src/sstable/footer.rs:86-131,
src/sstable/builder.rs:139-162, src/sstable/reader.rs:116-170).
"""
import io
import struct

import numpy as np
import pytest

import keygen
import lsmbloom
from lsmbloom import sstable


def _block(oracle, keys, nb, k):
    data, offs = keygen.pack(keys)
    return oracle.serialize(oracle.build_var(data, offs, nb, k), nb, k)


def test_footer_roundtrip_and_magic():
    ft = sstable.Footer(1, 2, 3, 4, 5, 6)
    b = ft.encode()
    assert len(b) == sstable.FOOTER_SIZE == 56
    assert struct.unpack("<7Q", b)[6] == 0x4C534D5F53535400
    assert vars(sstable.Footer.decode(b)) == vars(ft)
    with pytest.raises(lsmbloom.Corruption):
        sstable.Footer.decode(b[:55])
    bad = b[:48] + struct.pack("<Q", 0x1234)
    with pytest.raises(lsmbloom.Corruption, match="bad magic"):
        sstable.Footer.decode(bad)


def test_meta_block_roundtrip():
    m = sstable.encode_meta_block(42, b"apple", b"zebra!", 1000)
    assert len(m) == 8 + 4 + 4 + 5 + 4 + 6 + 8
    got = sstable.parse_meta_block(m)
    assert got == {"id": 42, "level": 0, "min_key": b"apple", "max_key": b"zebra!", "entry_count": 1000}
    with pytest.raises(lsmbloom.Corruption):
        sstable.parse_meta_block(m[:-3])


def test_index_entry_encoding():
    e = sstable.encode_index_entry(b"key_9", 4096, 123)
    assert e == struct.pack("<H", 5) + b"key_9" + struct.pack("<QQ", 4096, 123)


def test_bloom_block_between_meta_and_index(oracle, tmp_path):
    """footer_has_bloom_block_info (bloom_sstable_integration_tests.rs:142-174)
    on a file laid out by write_tail, then the block read back is the same
    filter (SSTable::open -> deserialize, reader.rs:78-82)."""
    nb, k = lsmbloom.params(1000, 0.01)  # SSTableBuilder::new sizing (builder.rs:51,74)
    keys = [b"key"]
    block = _block(oracle, keys, nb, k)
    path = tmp_path / "t.sst"
    data_blocks = b"\x00" * 77  # stands in for the encoded data block(s)
    with open(path, "wb") as f:
        f.write(data_blocks)
        sstable.write_tail(f, len(data_blocks), 1, b"key", b"key", 1, np.frombuffer(block, np.uint8),
                           sstable.encode_index_entry(b"key", 0, 77))
    ft, bloom, meta = sstable.read_tail(path)
    assert ft.bloom_block_size > 0 and ft.bloom_block_offset > 0
    assert ft.bloom_block_offset >= ft.meta_block_offset + ft.meta_block_size
    assert ft.bloom_block_offset + ft.bloom_block_size <= ft.index_block_offset
    assert bytes(bloom) == bytes(block)
    assert meta["min_key"] == b"key" and meta["entry_count"] == 1
    f2 = lsmbloom.BloomFilter.deserialize(bloom)
    assert f2.may_contain(b"key") and f2.num_bits() == nb and f2.num_hashes() == k


def test_read_tail_rejects_short_file(tmp_path):
    p = tmp_path / "short.sst"
    p.write_bytes(b"\x01" * 20)
    with pytest.raises(lsmbloom.Corruption, match="too short"):
        sstable.read_tail(p)


def test_key_arena_packs_like_builder():
    a = sstable.KeyArena()
    for kk in (b"a", b"", b"ccc"):
        a.add(kk)
    data, offs = a.arrays()
    assert len(a) == 3 and bytes(data) == b"accc" and offs.tolist() == [0, 1, 1, 4]
