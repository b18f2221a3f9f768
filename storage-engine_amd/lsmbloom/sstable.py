"""The SSTable bloom block on disk: the slice of SSTableBuilder::finish and
SSTable::open that touches src/bloom.

Write side (SSTableBuilder::finish, src/sstable/builder.rs:164-203): after the
data blocks come the meta block, the bloom block, the index block and the
56-byte footer.  Here the bloom block is produced by ONE GPU call
(lsmb_build_block: build + serialize, words copied device -> block), instead of
`bloom_builder.build()` + `bloom.serialize()` (builder.rs:177-179).

Read side (SSTable::open, src/sstable/reader.rs:56-110): footer -> bloom block ->
BloomFilter::deserialize (reader.rs:78-82).  `load_filter` hands the block to a
device-resident FilterSet (lsmb_fset_add validates it exactly like deserialize
and copies it straight into HBM) together with the table's [min_key, max_key]
from the meta block, so DB::get's per-table checks (reader.rs:192-199) run as
one batched GPU probe.

Data blocks and the index entries' content are the SST builder's business and
out of scope: callers pass the data-block end offset and the encoded index.
"""
import io
import os
import struct

import numpy as np

from . import Corruption, default_context, params

SSTABLE_MAGIC = 0x4C534D5F53535400  # "LSM_SST\0", src/sstable/footer.rs:6
FOOTER_SIZE = 8 * 7                 # footer.rs:84


class Footer:
    """src/sstable/footer.rs:72-146: seven LE u64 in this order."""

    FIELDS = ("index_block_offset", "index_block_size", "meta_block_offset", "meta_block_size",
              "bloom_block_offset", "bloom_block_size", "magic")

    def __init__(self, index_block_offset, index_block_size, meta_block_offset, meta_block_size,
                 bloom_block_offset, bloom_block_size, magic=SSTABLE_MAGIC):
        self.index_block_offset = index_block_offset
        self.index_block_size = index_block_size
        self.meta_block_offset = meta_block_offset
        self.meta_block_size = meta_block_size
        self.bloom_block_offset = bloom_block_offset
        self.bloom_block_size = bloom_block_size
        self.magic = magic

    def encode(self):  # footer.rs:86-96
        return struct.pack("<7Q", *(getattr(self, f) for f in self.FIELDS))

    @classmethod
    def decode(cls, data):  # footer.rs:98-131
        if len(data) < FOOTER_SIZE:
            raise Corruption(-4, "footer too short")
        vals = struct.unpack("<7Q", bytes(data[:FOOTER_SIZE]))
        if vals[6] != SSTABLE_MAGIC:
            raise Corruption(-4, "bad magic: expected %#x, got %#x" % (SSTABLE_MAGIC, vals[6]))
        return cls(*vals)


def encode_meta_block(sst_id, min_key, max_key, entry_count):
    """SSTableBuilder::encode_meta_block (builder.rs:139-162):
    [id u64][level u32 = 0][min_len u32][min_key][max_len u32][max_key][entry_count u64]."""
    min_key, max_key = bytes(min_key), bytes(max_key)
    return (struct.pack("<QII", sst_id, 0, len(min_key)) + min_key + struct.pack("<I", len(max_key)) + max_key
            + struct.pack("<Q", entry_count))


def parse_meta_block(buf):
    """SSTable::parse_meta (reader.rs, format comment at :88): -> dict."""
    buf = bytes(buf)
    try:
        sst_id, level, lmin = struct.unpack_from("<QII", buf, 0)
        p = 16
        min_key = buf[p:p + lmin]
        p += lmin
        (lmax,) = struct.unpack_from("<I", buf, p)
        p += 4
        max_key = buf[p:p + lmax]
        p += lmax
        (count,) = struct.unpack_from("<Q", buf, p)
    except struct.error as e:
        raise Corruption(-4, "meta block truncated: %s" % e)
    if len(min_key) != lmin or len(max_key) != lmax:
        raise Corruption(-4, "meta block truncated")
    return {"id": sst_id, "level": level, "min_key": min_key, "max_key": max_key, "entry_count": count}


def encode_index_entry(last_key, offset, size):
    """IndexEntry::encode (footer.rs:20-27): [key_len u16][last_key][offset u64][size u64]."""
    last_key = bytes(last_key)
    return struct.pack("<H", len(last_key)) + last_key + struct.pack("<QQ", offset, size)


class KeyArena:
    """BloomFilterBuilder's key buffer (one SST's keys, packed + offsets).  The
    reference inserts per key at SSTableBuilder::add (builder.rs:93); the arena
    defers every insert to the one GPU build at finish."""

    def __init__(self):
        self._buf = io.BytesIO()
        self._offs = [0]

    def add(self, key):
        self._buf.write(bytes(key))
        self._offs.append(self._buf.tell())

    def __len__(self):
        return len(self._offs) - 1

    def arrays(self):
        return (np.frombuffer(self._buf.getbuffer(), dtype=np.uint8).copy(),
                np.array(self._offs, dtype=np.uint64))


def build_bloom_block(data, offsets, num_bits, k, ctx=None, key_len=0):
    """The bloom block bytes (BloomFilter::serialize of the filter built over the
    keys) from one lsmb_build_block call; `offsets` None selects fixed key_len keys."""
    ctx = ctx or default_context()
    return ctx.build_block(data, num_bits, k, offsets=offsets, key_len=key_len)


def write_tail(f, data_end, sst_id, min_key, max_key, entry_count, bloom_block, index_block):
    """SSTableBuilder::finish steps 2-5 (builder.rs:168-203) at file offset
    data_end (the end of the last data block): meta, bloom, index, footer.
    Returns the Footer.  `f` is a binary file object positioned at data_end."""
    meta = encode_meta_block(sst_id, min_key, max_key, entry_count)
    meta_off = data_end
    f.write(meta)
    bloom_off = meta_off + len(meta)
    bb = memoryview(np.ascontiguousarray(np.frombuffer(bloom_block, dtype=np.uint8)))  # no copy of the words
    f.write(bb)
    bloom_size = bb.nbytes
    index_off = bloom_off + bloom_size
    index_block = bytes(index_block)
    f.write(index_block)
    ft = Footer(index_off, len(index_block), meta_off, len(meta), bloom_off, bloom_size)
    f.write(ft.encode())
    return ft


def finish_sstable(path, data_blocks, sst_id, keys, index_block, fpr=0.01, expected_keys=1000, ctx=None):
    """Writes one SSTable tail the way SSTableBuilder::finish does, with the bloom
    block built on the GPU.  data_blocks: bytes already encoded by the SST
    builder (written first); keys: KeyArena of the table's keys in order (min =
    first, max = last, as builder.rs tracks them); the filter is sized
    BloomFilter::new(expected_keys, fpr) like SSTableBuilder::new /
    with_estimated_keys (builder.rs:51,74).  Returns the Footer."""
    nb, k = params(max(expected_keys, 1), fpr)  # builder.rs:74
    data, offs = keys.arrays()
    block = build_bloom_block(data, offs, nb, k, ctx=ctx)
    n = len(keys)
    min_key = bytes(data[int(offs[0]):int(offs[1])]) if n else b""
    max_key = bytes(data[int(offs[n - 1]):int(offs[n])]) if n else b""
    with open(path, "wb") as f:
        f.write(bytes(data_blocks))
        ft = write_tail(f, len(data_blocks), sst_id, min_key, max_key, n, block, index_block)
        f.flush()
        os.fsync(f.fileno())  # builder.rs:199-200
    return ft


def read_tail(path):
    """SSTable::open's footer / bloom / meta reads (reader.rs:56-110) ->
    (Footer, bloom block bytes, meta dict).  Corruption as the reference."""
    with open(path, "rb") as f:
        f.seek(0, os.SEEK_END)
        size = f.tell()
        if size < FOOTER_SIZE:
            raise Corruption(-4, "file too short to contain footer")
        f.seek(size - FOOTER_SIZE)
        ft = Footer.decode(f.read(FOOTER_SIZE))
        f.seek(ft.bloom_block_offset)
        bloom = f.read(ft.bloom_block_size)
        f.seek(ft.meta_block_offset)
        meta_buf = f.read(ft.meta_block_size)
    if len(bloom) != ft.bloom_block_size:
        raise Corruption(-4, "bloom block truncated")
    meta = parse_meta_block(meta_buf) if meta_buf else {"id": 0, "level": 0, "min_key": b"", "max_key": b"",
                                                        "entry_count": 0}
    return ft, bloom, meta


def load_filter(fset, path):
    """SSTable::open's bloom load (reader.rs:78-82) into a device-resident
    FilterSet with the table's key range; returns the slot."""
    _, bloom, meta = read_tail(path)
    return fset.add(bloom, meta["min_key"], meta["max_key"])
