"""Pins the CPU oracle (oracle/bloom_oracle.c) to the golden fixtures.

The fixtures come from tests/golden/gen_golden.py (Python xxhash 0.8.2 cross-checked
with system libxxhash 0.8.1, plus a pure-Python restatement of src/bloom/mod.rs that
replays the reference tests' deterministic assertions).  CPU only.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import keygen

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _j(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


XXH = _j("xxh3_vectors.json")
KATS = _j("bloom_kats.json")
C1 = _j("c1_fixture.json")
VAR = _j("varlen_fixture.json")


def test_xxh3_every_length_class(oracle):
    for v in XXH["vectors"]:
        lo, hi = oracle.xxh3_128(bytes.fromhex(v["input"]))
        assert (lo, hi) == (int(v["lo"], 16), int(v["hi"], 16)), v["len"]


def test_xxh3_known_answers(oracle):
    # SURVEY §8c KATs: xxh3_128(b"") and xxh3_128(b"hello")
    assert oracle.xxh3_128(b"") == (0x6001C324468D497F, 0x99AA06D3014798D8)
    assert oracle.xxh3_128(b"hello") == (0xC779CFAA5E523818, 0xB5E9C1AD071B3E7F)
    z = XXH["zeros_1mib"]
    assert oracle.xxh3_128(bytes(1 << 20)) == (int(z["lo"], 16), int(z["hi"], 16))


def test_sizing_table(oracle):
    for s in KATS["sizing"]:
        assert oracle.params(s["n"], s["fpr"]) == (s["num_bits"], s["k"]), s


def test_sizing_panics(oracle):
    # BloomFilter::new asserts (src/bloom/mod.rs:39-43)
    for n, fpr in ((0, 0.01), (10, 0.0), (10, 1.0), (10, -0.5), (10, float("nan"))):
        with pytest.raises(ValueError):
            oracle.params(n, fpr)


def test_positions(oracle):
    for p in KATS["positions"] + KATS["raw_positions"]:
        assert oracle.positions(bytes.fromhex(p["key"]), p["num_bits"], p["k"]) == p["positions"]


def test_reference_scenarios(oracle):
    for sc in KATS["scenarios"]:
        nb, k = oracle.params(sc["n"], sc["fpr"])
        assert (nb, k) == (sc["num_bits"], sc["k"])
        w = np.zeros(oracle.nwords(nb), np.uint64)
        for key in sc["inserts"]:
            oracle.insert(w, nb, k, bytes.fromhex(key))
        for key, expect in sc["probes"]:
            assert oracle.may_contain(w, nb, k, bytes.fromhex(key)) == expect, (sc["name"], key)
        ser = oracle.serialize(w, nb, k)
        assert hashlib.sha256(ser).hexdigest() == sc["serialized_sha256"], sc["name"]
        if "serialized_hex" in sc:
            assert ser.hex() == sc["serialized_hex"]


def _fmt_keys(c):
    name = c["name"]
    if name == "false_positive_rate":
        return ([b"key_%d" % i for i in range(10000)], [b"key_%d" % i for i in range(10000, 20000)])
    if name.startswith("various_fpr_"):
        d = c["desc"]
        return ([("test_%s_%d" % (d, i)).encode() for i in range(5000)],
                [("test_%s_%d" % (d, i)).encode() for i in range(5000, 10000)])
    if name == "sstable_exist_fpr":
        return ([b"exist_%06d" % i for i in range(1000)], [b"exist_%06d" % i for i in range(1000, 11000)])
    if name == "large_key_1mib_zeros":
        return ([bytes(1 << 20)], [bytes(1 << 20)])
    raise KeyError(name)


def test_reference_fpr_counts(oracle):
    for c in KATS["counts"]:
        ins, probes = _fmt_keys(c)
        nb, k = oracle.params(c["n"], c["fpr"])
        d, o = keygen.pack(ins)
        w = oracle.build_var(d, o, nb, k)
        ser = oracle.serialize(w, nb, k)
        assert hashlib.sha256(ser).hexdigest() == c["serialized_sha256"], c["name"]
        pd, po = keygen.pack(probes)
        m = oracle.probe([(w, nb, k)], pd, po)
        assert m[:len(ins)].all() if c["name"] == "large_key_1mib_zeros" else True
        if "false_positives" in c:
            assert int(m.sum()) == c["false_positives"], c["name"]
            # the reference bands (bloom_tests.rs:94-109, :138-146)
            assert c["false_positives"] / len(probes) < 3 * c["fpr"]
        # no false negatives
        mm = oracle.probe([(w, nb, k)], d, o)
        assert mm.all()


def test_c1_fixture(oracle):
    keys = keygen.key16(0x5EED0001, 0, C1["n"])
    assert keys[0].tobytes().hex() == C1["first_key"]
    assert np.array_equal(keys, oracle.key16(0x5EED0001, 0, C1["n"]))
    nb, k = oracle.params(C1["n"], 0.01)
    assert (nb, k) == (C1["num_bits"], C1["k"])
    w = oracle.build_fixed(keys, 16, nb, k)
    ser = oracle.serialize(w, nb, k)
    assert hashlib.sha256(ser).hexdigest() == C1["serialized_sha256"]
    assert int(np.unpackbits(w.view(np.uint8)).sum()) == C1["popcount"]
    assert [f"{x:016x}" for x in w[:16]] == C1["first_words"]
    nm = keygen.key16(0x5EED0002, 0, C1["n"])
    m = oracle.probe([(w, nb, k)], nm, key_len=16)
    assert int(m.sum()) == C1["nonmember_false_positives"]
    assert hashlib.sha256(m.reshape(-1).tobytes()).hexdigest() == C1["nonmember_probe_sha256"]
    # multi-threaded baseline gives identical bits
    w2 = oracle.build_fixed_mt(keys, 16, nb, k, 4)
    assert np.array_equal(w, w2)


def test_varlen_fixture(oracle):
    data, offs = keygen.varlen(VAR["n"])
    assert hashlib.sha256(data.tobytes()).hexdigest() == VAR["data_sha256"]
    assert [int(x) for x in np.diff(offs[:17])] == VAR["first_lengths"]
    nb, k = oracle.params(VAR["n"], 0.01)
    w = oracle.build_var(data, offs, nb, k)
    assert hashlib.sha256(oracle.serialize(w, nb, k)).hexdigest() == VAR["serialized_sha256"]
    nm = keygen.key16(0x5EED0002, 0, VAR["n"])
    m = oracle.probe([(w, nb, k)], nm, key_len=16)
    assert int(m.sum()) == VAR["nonmember_false_positives"]


def test_deserialize_validation(oracle):
    # bloom_serialize_tests.rs:61-92 and src/bloom/mod.rs:126-153
    for bad in (b"\xff\xff\xff\xff", b""):
        with pytest.raises(ValueError):
            oracle.deserialize(bad)
    trunc = (7).to_bytes(4, "little") + (1000).to_bytes(4, "little") + (100).to_bytes(4, "little")
    with pytest.raises(ValueError):
        oracle.deserialize(trunc)
    nb, k = oracle.params(10, 0.01)
    w = np.zeros(oracle.nwords(nb), np.uint64)
    oracle.insert(w, nb, k, b"test")
    ser = oracle.serialize(w, nb, k)
    with pytest.raises(ValueError):
        oracle.deserialize(ser + b"extra")
    k2, nb2, w2 = oracle.deserialize(ser)
    assert (k2, nb2) == (k, nb) and np.array_equal(w, w2)


def test_fullsize_fixture_fill_ratios(oracle):
    """The full-size digests (tests/golden/gen_fullsize.py) are plausible Bloom
    filters of their stated workloads: sizing as BloomFilter::new gives it,
    and the fill ratio within 1e-4 of 1 - exp(-k n / m) (its standard
    deviation here is ~1e-5)."""
    import math
    fx = json.load(open(os.path.join(GOLD, "fullsize_fixture.json")))
    work = {"c2": (10**8, 10**8), "c2_exact10": (10**8, None), "c4": (10**8, 10**8),
            "c5": (10**9, 10**9), "c5_shard0": (125_000_000, 10**9)}
    assert set(fx) == set(work)
    for name, (n, sized_for) in work.items():
        e = fx[name]
        if sized_for is None:
            assert (e["num_bits"], e["k"]) == (10 * n, 7)
        else:
            assert (e["num_bits"], e["k"]) == tuple(oracle.params(sized_for, 0.01)), name
        assert e["words"] == (e["num_bits"] + 63) // 64
        want = 1.0 - math.exp(-e["k"] * n / e["num_bits"])
        assert abs(e["popcount"] / e["num_bits"] - want) < 1e-4, name
