#!/usr/bin/env python3
"""Full-size word fixtures for the GPU build configs.

For C2 (canonical and exact 10 bits/key), C4 and C5 this builds the whole
filter with the CPU oracle (oracle/bloom_oracle.c, multithreaded, the same
bits as the reference's per-key insert loop: OR is order-independent) from
the BASELINE.md generators (tests/keygen.py, oracle_gen_key16), in chunks, and
records num_bits, k, popcount, the sha256 of the little-endian words and the
first/last 8 words.  tests/test_gpu_parity.py and bench.py compare the GPU's
full-size filters against these digests, so full-size parity no longer needs
the oracle at run time.

Run here (CPU): python3 tests/golden/gen_fullsize.py  (~2-4 min, ~3 GB RAM);
`gen_fullsize.py c5_shard0` adds or refreshes that entry alone.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import keygen  # noqa: E402
import oracle_ct  # noqa: E402

SEED_MEMBERS = 0x5EED0001
THREADS = os.cpu_count() or 8


def digest(words, nb, k, what):
    w = np.ascontiguousarray(words, dtype="<u8")
    return {"what": what, "num_bits": int(nb), "k": int(k), "words": int(w.size),
            "popcount": int(np.bitwise_count(w).sum()),
            "sha256": hashlib.sha256(w.tobytes()).hexdigest(),
            "first8": [int(x) for x in w[:8]], "last8": [int(x) for x in w[-8:]]}


def build_key16(orc, n, nb, k, chunk=50_000_000):
    words = np.zeros(orc.nwords(nb), dtype=np.uint64)
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        orc.build_fixed_mt(orc.key16(SEED_MEMBERS, first, m), 16, nb, k, THREADS, words=words)
    return words


def build_c4(orc, n, nb, k, chunk=10_000_000):
    words = np.zeros(orc.nwords(nb), dtype=np.uint64)
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        data, offs = keygen.varlen(m, first)
        orc.build_var_mt(data, offs, nb, k, THREADS, words=words)
    return words


def c5_shard0(orc):
    """The N = 8 per-GPU C5 build on one GPU (bench.py's c5_shard leg): the
    first 125 M C5 keys into new(1e9, 0.01) = 2^32-1 bits."""
    nb5, k5 = orc.params(1_000_000_000, 0.01)
    return digest(build_key16(orc, 125_000_000, nb5, k5), nb5, k5,
                  "C5 shard 0 of 8: key16(0x5EED0001, 0..1.25e8) into new(1e9, 0.01) = 2^32-1 bits")


def main():
    orc = oracle_ct.load()
    path = os.path.join(HERE, "fullsize_fixture.json")
    if sys.argv[1:] == ["c5_shard0"]:  # add / refresh that entry only (~1 min)
        out = json.load(open(path))
        out["c5_shard0"] = c5_shard0(orc)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return
    out = {}
    t0 = time.time()
    nb, k = orc.params(100_000_000, 0.01)
    out["c2"] = digest(build_key16(orc, 100_000_000, nb, k), nb, k,
                       "C2: key16(0x5EED0001, 0..1e8) into new(1e8, 0.01)")
    print("c2 %.0fs" % (time.time() - t0), flush=True)
    out["c2_exact10"] = digest(build_key16(orc, 100_000_000, 1_000_000_000, 7), 1_000_000_000, 7,
                               "C2 exact: the same keys into num_bits = 10 n = 1e9, k = 7")
    print("c2_exact10 %.0fs" % (time.time() - t0), flush=True)
    out["c4"] = digest(build_c4(orc, 100_000_000, nb, k), nb, k,
                       "C4: keygen.varlen(1e8) (8-256 B) into new(1e8, 0.01)")
    print("c4 %.0fs" % (time.time() - t0), flush=True)
    nb5, k5 = orc.params(1_000_000_000, 0.01)
    out["c5"] = digest(build_key16(orc, 1_000_000_000, nb5, k5), nb5, k5,
                       "C5: key16(0x5EED0001, 0..1e9) into new(1e9, 0.01) = 2^32-1 bits")
    print("c5 %.0fs" % (time.time() - t0), flush=True)
    out["c5_shard0"] = c5_shard0(orc)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
