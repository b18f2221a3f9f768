#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the build container only).

The reference (G1DO/Storage-Engine, Rust) cannot be compiled here (no cargo /
rustc, crates not vendored, no network).  Its hot path is `src/bloom/mod.rs`,
whose only arithmetic dependency is `xxhash_rust::xxh3::xxh3_128` (crate
xxhash-rust 0.8.15, `Cargo.lock:694-697`).  XXH3 output is frozen since xxHash
0.8.0, so the fixtures are produced from:

* the Python `xxhash` module (3.8.1, bundling libxxhash 0.8.2) for the hash,
  cross-checked bit-for-bit against the system `libxxhash.so.0.8.1` via ctypes;
* a pure-Python restatement of `src/bloom/mod.rs` (sizing :38-67, hash split
  :181-189, positions :192-197, bit layout :200-211, format :102-115) below.

The restatement is itself pinned by replaying the deterministic assertions of
the reference's tests (tests/bloom_tests.rs, tests/bloom_serialize_tests.rs,
tests/bloom_sstable_integration_tests.rs); `check_reference_assertions()` fails
loudly if any of them does not hold.

Outputs (data only — inputs and expected outputs):
  xxh3_vectors.json   hash vectors for every length class
  bloom_kats.json     sizing table, positions, per-test scenarios, serialized filters
  c1_fixture.json     BASELINE config C1 (100k key16) filter + probe digests
  varlen_fixture.json C4-shaped var-len keys (first 20k) filter digest

Usage:  python3 tests/golden/gen_golden.py
"""
import ctypes
import hashlib
import json
import math
import os
import struct

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1


# --------------------------------------------------------------------------- hash
def xxh3_128(b: bytes):
    """(h1, h2) = (low64, high64) of xxh3_128(key), seed 0 (src/bloom/mod.rs:181-189)."""
    d = xxhash.xxh3_128_intdigest(b)
    return d & M64, d >> 64


class _U128(ctypes.Structure):
    _fields_ = [("low64", ctypes.c_uint64), ("high64", ctypes.c_uint64)]


def _libxxhash():
    for name in ("libxxhash.so.0", "/usr/lib/x86_64-linux-gnu/libxxhash.so.0.8.1"):
        try:
            lib = ctypes.CDLL(name)
            lib.XXH3_128bits.restype = _U128
            lib.XXH3_128bits.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
            return lib
        except OSError:
            continue
    return None


# --------------------------------------------------------------------------- generators
def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def key16(seed, i):
    """BASELINE.md key generator: LE64(sm(seed+2i)) || LE64(sm(seed+2i+1))."""
    return struct.pack("<QQ", splitmix64(seed + 2 * i), splitmix64(seed + 2 * i + 1))


def stream_bytes(seed, off, n):
    """Byte o of the stream = byte (o % 8) of LE64(sm(seed + o // 8))."""
    out = bytearray()
    w0 = off // 8
    w1 = (off + n + 7) // 8
    for w in range(w0, w1):
        out += struct.pack("<Q", splitmix64(seed + w))
    s = off - w0 * 8
    return bytes(out[s:s + n])


VAR_LEN_SEED = 0x5EED0003   # len_i = 8 + sm(VAR_LEN_SEED + i) % 249
VAR_DATA_SEED = 0x5EED0004  # packed data = stream_bytes(VAR_DATA_SEED, 0, total)


def varlen_keys(n):
    lens = [8 + splitmix64(VAR_LEN_SEED + i) % 249 for i in range(n)]
    offs = [0]
    for L in lens:
        offs.append(offs[-1] + L)
    data = stream_bytes(VAR_DATA_SEED, 0, offs[-1])
    return data, offs


# --------------------------------------------------------------------------- src/bloom restatement
def sat_u32(x):
    if x != x or x <= 0:
        return 0
    if x >= 4294967295.0:
        return 4294967295
    return int(x)


def bloom_params(n, fpr):
    """BloomFilter::new sizing, src/bloom/mod.rs:38-67."""
    assert n > 0 and 0.0 < fpr < 1.0
    bpk = -1.44 * math.log2(fpr)
    nb = max(sat_u32(math.ceil(float(n) * bpk)), 64)
    k = max(sat_u32(math.ceil(bpk * math.log(2.0))), 1)
    return nb, k


class Bloom:
    """Pure-Python restatement of src/bloom/mod.rs:23-211."""

    def __init__(self, n=None, fpr=None, num_bits=None, k=None):
        if num_bits is None:
            num_bits, k = bloom_params(n, fpr)
        self.num_bits, self.k = num_bits, k
        self.words = [0] * ((num_bits + 63) // 64)

    def positions(self, key):
        h1, h2 = xxh3_128(key)
        return [((h1 + i * h2) & M64) % self.num_bits for i in range(self.k)]

    def insert(self, key):
        for p in self.positions(key):
            self.words[p // 64] |= 1 << (p % 64)

    def may_contain(self, key):
        return all((self.words[p // 64] >> (p % 64)) & 1 for p in self.positions(key))

    def serialize(self):
        return struct.pack("<III", self.k, self.num_bits, len(self.words)) + b"".join(
            struct.pack("<Q", w) for w in self.words)

    def popcount(self):
        return sum(bin(w).count("1") for w in self.words)


def sha(b):
    return hashlib.sha256(b).hexdigest()


# --------------------------------------------------------------------------- reference assertions
def check_reference_assertions():
    """Replays the deterministic assertions of the reference's bloom tests."""
    bf = Bloom(100, 0.01)
    assert not bf.may_contain(b"any_key") and not bf.may_contain(b"hello") and not bf.may_contain(b"")
    bf.insert(b"hello")                                  # bloom_tests.rs:14-34
    assert bf.may_contain(b"hello")
    for k in (b"world", b"hello!", b"hell"):
        assert not bf.may_contain(k), k
    bf = Bloom(100, 0.01)                               # bloom_tests.rs:50-65
    for k in (b"apple", b"banana", b"cherry"):
        bf.insert(k)
    assert not bf.may_contain(b"date") and not bf.may_contain(b"elderberry")
    bf = Bloom(100, 0.01)                               # bloom_tests.rs:170-181
    bf.insert(bytes([0, 1, 2, 0xFF, 0xFE]))
    assert not bf.may_contain(bytes([0xFF, 0xFE, 0xFD, 0xFC]))
    bf = Bloom(100, 0.01)                               # bloom_serialize_tests.rs:4-26
    for k in (b"hello", b"world", b"foo"):
        bf.insert(k)
    assert not bf.may_contain(b"bar") and not bf.may_contain(b"baz")
    bf = Bloom(100, 0.01)                               # bloom_serialize_tests.rs:127-141
    bf.insert(bytes([0, 1, 2, 0xFF]))
    assert not bf.may_contain(bytes([0xFF, 0xFE, 0xFD, 0xFC]))


# --------------------------------------------------------------------------- fixtures
def gen_xxh3(lib):
    vecs = []
    lengths = list(range(0, 301)) + [511, 512, 513, 1023, 1024, 1025, 1026, 2047, 2048, 2049, 4096]
    for L in lengths:
        data = stream_bytes(0xA11CE + L * 7919, 0, L)
        lo, hi = xxh3_128(data)
        if lib is not None:
            r = lib.XXH3_128bits(data, len(data))
            assert (r.low64, r.high64) == (lo, hi), L
        vecs.append({"len": L, "input": data.hex(), "lo": f"{lo:016x}", "hi": f"{hi:016x}"})
    z = bytes(1 << 20)
    lo, hi = xxh3_128(z)
    if lib is not None:
        r = lib.XXH3_128bits(z, len(z))
        assert (r.low64, r.high64) == (lo, hi)
    return {
        "source": "python xxhash %s (libxxhash %s), cross-checked vs system libxxhash.so.0.8.1: %s"
                  % (xxhash.VERSION, xxhash.XXHASH_VERSION, lib is not None),
        "input_rule": "input of length L = stream_bytes(0xA11CE + 7919*L, 0, L); stored hex",
        "vectors": vecs,
        "zeros_1mib": {"len": 1 << 20, "lo": f"{lo:016x}", "hi": f"{hi:016x}"},
    }


def scenario(name, cite, n, fpr, inserts, probes, keep_hex=True):
    bf = Bloom(n, fpr)
    for k in inserts:
        bf.insert(k)
    ser = bf.serialize()
    d = {
        "name": name, "cite": cite, "n": n, "fpr": fpr,
        "num_bits": bf.num_bits, "k": bf.k,
        "inserts": [k.hex() for k in inserts],
        "probes": [[k.hex(), bool(bf.may_contain(k))] for k in probes],
        "serialized_sha256": sha(ser), "serialized_len": len(ser), "popcount": bf.popcount(),
    }
    if keep_hex and len(ser) <= 2048:
        d["serialized_hex"] = ser.hex()
    return d


def gen_kats():
    sizing = []
    for n in (1, 2, 10, 44, 45, 100, 1000, 5000, 10000, 100000, 10**6, 10**8, 10**9,
              2**32, 10**10):
        for fpr in (0.5, 0.1, 0.05, 0.01, 0.001, 1e-6):
            nb, k = bloom_params(n, fpr)
            sizing.append({"n": n, "fpr": fpr, "num_bits": nb, "k": k})
    positions = []
    for (n, fpr) in ((100, 0.01), (1000, 0.01), (10**8, 0.01), (10**9, 0.01), (5000, 0.001)):
        bf = Bloom(n, fpr)
        for key in (b"hello", b"", b"a", b"key_00000", bytes(range(16)), bytes(200)):
            positions.append({"n": n, "fpr": fpr, "num_bits": bf.num_bits, "k": bf.k,
                              "key": key.hex(), "positions": bf.positions(key)})
    # exhaustive-modulus probes: positions at extreme num_bits via raw (num_bits, k)
    raw = []
    for nb in (64, 65, 957, 9568, 956716, 956715292, 2**31, 2**31 + 1, 4294967295):
        bf = Bloom(num_bits=nb, k=13)
        for i in range(64):
            key = key16(0xC0FFEE, i)
            raw.append({"num_bits": nb, "k": 13, "key": key.hex(), "positions": bf.positions(key)})

    sc = []
    sc.append(scenario("empty_filter_returns_false", "tests/bloom_tests.rs:4-11", 100, 0.01, [],
                       [b"any_key", b"hello", b""]))
    sc.append(scenario("inserted_and_different", "tests/bloom_tests.rs:14-34", 100, 0.01, [b"hello"],
                       [b"hello", b"world", b"hello!", b"hell"]))
    sc.append(scenario("duplicate_insert", "tests/bloom_tests.rs:37-47", 100, 0.01, [b"key"] * 3, [b"key"]))
    sc.append(scenario("multiple_keys", "tests/bloom_tests.rs:50-65", 100, 0.01,
                       [b"apple", b"banana", b"cherry"],
                       [b"apple", b"banana", b"cherry", b"date", b"elderberry"]))
    sc.append(scenario("empty_key", "tests/bloom_tests.rs:151-157", 100, 0.01, [b""], [b""]))
    sc.append(scenario("binary_keys", "tests/bloom_tests.rs:170-181", 100, 0.01,
                       [bytes([0, 1, 2, 0xFF, 0xFE])],
                       [bytes([0, 1, 2, 0xFF, 0xFE]), bytes([0xFF, 0xFE, 0xFD, 0xFC])]))
    sc.append(scenario("serialize_roundtrip", "tests/bloom_serialize_tests.rs:4-26", 100, 0.01,
                       [b"hello", b"world", b"foo"],
                       [b"hello", b"world", b"foo", b"bar", b"baz"]))
    sc.append(scenario("serialize_extra_data_src", "tests/bloom_serialize_tests.rs:84-92", 10, 0.01,
                       [b"test"], [b"test"]))
    for fpr in (0.1, 0.05, 0.01, 0.001):
        sc.append(scenario("serialize_different_fpr_%g" % fpr, "tests/bloom_serialize_tests.rs:113-124",
                           1000, fpr, [b"test_key"], [b"test_key"]))
    sc.append(scenario("serialize_binary_keys", "tests/bloom_serialize_tests.rs:127-141", 100, 0.01,
                       [bytes([0, 1, 2, 0xFF])], [bytes([0, 1, 2, 0xFF]), bytes([0xFF, 0xFE, 0xFD, 0xFC])]))
    sc.append(scenario("sstable_key_00000_00099", "tests/bloom_sstable_integration_tests.rs:12-33 "
                       "(SSTableBuilder::new sizing = new(1000, 0.01), src/sstable/builder.rs:51,74)",
                       1000, 0.01, [b"key_%05d" % i for i in range(100)],
                       [b"key_%05d" % i for i in range(100, 200)]))

    # FPR-count scenarios (digests only; the probe lists are regenerated by rule)
    counts = []
    bf = Bloom(10000, 0.01)                                   # bloom_tests.rs:68-110
    for i in range(10000):
        bf.insert(b"key_%d" % i)
    fp = sum(bf.may_contain(b"key_%d" % i) for i in range(10000, 20000))
    counts.append({"name": "false_positive_rate", "cite": "tests/bloom_tests.rs:68-110",
                   "n": 10000, "fpr": 0.01, "insert_rule": "key_{i} for i in 0..10000",
                   "probe_rule": "key_{i} for i in 10000..20000", "false_positives": fp,
                   "serialized_sha256": sha(bf.serialize()), "popcount": bf.popcount()})
    for fpr, desc in ((0.10, "10%"), (0.05, "5%"), (0.01, "1%"), (0.001, "0.1%")):  # :113-148
        bf = Bloom(5000, fpr)
        for i in range(5000):
            bf.insert(("test_%s_%d" % (desc, i)).encode())
        fp = sum(bf.may_contain(("test_%s_%d" % (desc, i)).encode()) for i in range(5000, 10000))
        counts.append({"name": "various_fpr_%s" % desc, "cite": "tests/bloom_tests.rs:113-148",
                       "n": 5000, "fpr": fpr, "insert_rule": "test_{desc}_{i} for i in 0..5000",
                       "desc": desc, "probe_rule": "test_{desc}_{i} for i in 5000..10000",
                       "false_positives": fp, "serialized_sha256": sha(bf.serialize()),
                       "popcount": bf.popcount()})
    bf = Bloom(1000, 0.01)                                    # integration :66-113
    for i in range(1000):
        bf.insert(b"exist_%06d" % i)
    fp = sum(bf.may_contain(b"exist_%06d" % i) for i in range(1000, 11000))
    counts.append({"name": "sstable_exist_fpr", "cite": "tests/bloom_sstable_integration_tests.rs:66-113",
                   "n": 1000, "fpr": 0.01, "insert_rule": "exist_{i:06} for i in 0..1000",
                   "probe_rule": "exist_{i:06} for i in 1000..11000", "false_positives": fp,
                   "serialized_sha256": sha(bf.serialize()), "popcount": bf.popcount()})
    big = Bloom(100, 0.01)                                    # bloom_tests.rs:160-167
    big.insert(bytes(1 << 20))
    counts.append({"name": "large_key_1mib_zeros", "cite": "tests/bloom_tests.rs:160-167",
                   "n": 100, "fpr": 0.01, "insert_rule": "one key of 1 MiB zero bytes",
                   "serialized_sha256": sha(big.serialize()), "popcount": big.popcount(),
                   "serialized_hex": big.serialize().hex()})
    return {"sizing": sizing, "positions": positions, "raw_positions": raw,
            "scenarios": sc, "counts": counts}


def gen_c1():
    n = 100000
    bf = Bloom(n, 0.01)
    for i in range(n):
        bf.insert(key16(0x5EED0001, i))
    probe = bytes(int(bf.may_contain(key16(0x5EED0002, i))) for i in range(n))
    ser = bf.serialize()
    return {"config": "C1: new(100000, 0.01), members key16(0x5EED0001, i), non-members key16(0x5EED0002, i)",
            "n": n, "num_bits": bf.num_bits, "k": bf.k, "popcount": bf.popcount(),
            "serialized_sha256": sha(ser), "serialized_len": len(ser),
            "first_key": key16(0x5EED0001, 0).hex(),
            "nonmember_false_positives": sum(probe), "nonmember_probe_sha256": sha(probe),
            "first_words": [f"{w:016x}" for w in bf.words[:16]],
            "last_words": [f"{w:016x}" for w in bf.words[-16:]]}


def gen_varlen():
    n = 20000
    data, offs = varlen_keys(n)
    bf = Bloom(n, 0.01)
    for i in range(n):
        bf.insert(data[offs[i]:offs[i + 1]])
    # probe: members 0..n and non-members = 16-byte key16(0x5EED0002, i)
    nm = bytes(int(bf.may_contain(key16(0x5EED0002, i))) for i in range(n))
    return {"config": "C4 shape: len_i = 8 + sm(0x5EED0003+i) % 249; data byte o = byte o%8 of "
                      "LE64(sm(0x5EED0004 + o//8)); first 20000 keys into new(20000, 0.01)",
            "n": n, "total_bytes": offs[-1], "num_bits": bf.num_bits, "k": bf.k,
            "first_lengths": [offs[i + 1] - offs[i] for i in range(16)],
            "data_sha256": sha(data), "popcount": bf.popcount(),
            "serialized_sha256": sha(bf.serialize()),
            "nonmember_false_positives": sum(nm), "nonmember_probe_sha256": sha(nm)}


def main():
    check_reference_assertions()
    lib = _libxxhash()
    out = {
        "xxh3_vectors.json": gen_xxh3(lib),
        "bloom_kats.json": gen_kats(),
        "c1_fixture.json": gen_c1(),
        "varlen_fixture.json": gen_varlen(),
    }
    for name, obj in out.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
