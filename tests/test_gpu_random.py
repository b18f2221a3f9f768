"""Randomized GPU parity sweep (seeded, reproducible).

Each case draws a filter size log-uniformly over 2^6 .. 2^31 bits (so every
build strategy shows up: whole-filter LDS, tiled, atomic, partition with one or
several sweeps), k in 1..40 (k > 32 takes the atomic strategy), a batch size
log-uniformly over 1 .. ~3 M keys, and a key shape: 16-B keys, random fixed
lengths 1..64 B (length 1: only 256 distinct keys, so heavy duplicates and the
partition's region-overflow path), or variable lengths 0..300 B (the empty key
included).  The device build OR-accumulates into words with a sparse preset
pattern, and every word must equal the oracle's build from the same preset;
then members + fresh keys are probed and every answer must equal the oracle's
may_contain (src/bloom/mod.rs:70-94).  The oracle is the checker only.
"""
import numpy as np
import pytest

import keygen
import lsmbloom

pytestmark = pytest.mark.gpu

CASES = 54
THREADS = 8


@pytest.fixture(scope="module")
def ctx():
    c = lsmbloom.Context(0)
    yield c
    c.close()


def draw(i):
    """Case i: key shape i % 3 x size band (i // 3) % 3, three draws of each pair.
    Bands: 2^6..2^21 bits (whole-filter LDS / tiled), 2^21..2^27 (tiled /
    atomic / small partitions), 2^27..2^31 (partition, one or more sweeps)."""
    rng = np.random.default_rng(0xB1005EED + i)
    lo, hi = ((6, 21), (21, 27), (27, 31))[(i // 3) % 3]
    nb = int(max(64, min(2**31, round(2.0 ** rng.uniform(lo, hi)))))
    k = 7 if rng.random() < 0.4 else int(rng.integers(1, 41))
    shape = ("fixed16", "fixedn", "var")[i % 3]
    n = int(2.0 ** rng.uniform(0, 21.5))
    if lo >= 27:  # big filters: enough keys that the partitioned path runs
        n = max(n, nb // 64)
    n = min(n, 300_000 if shape == "var" else 3_000_000)
    return rng, nb, k, shape, n


def keys_for(rng, shape, n, seed):
    """(data, offsets or None, key_len) for n keys of the given shape."""
    if shape == "fixed16":
        return keygen.key16(seed, 0, n).reshape(-1), None, 16
    if shape == "fixedn":
        L = int(rng.integers(1, 65))
        return rng.integers(0, 256, size=n * L, dtype=np.uint8), None, L
    lens = rng.integers(0, 301, size=n, dtype=np.uint64)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8), offs, 0


@pytest.mark.parametrize("case", range(CASES))
def test_random_build_and_probe_vs_oracle(ctx, oracle, case):
    rng, nb, k, shape, n = draw(case)
    data, offs, key_len = keys_for(rng, shape, n, 0x5EED7000 + case)
    preset = np.zeros(lsmbloom.num_words(nb), dtype=np.uint64)
    hot = rng.integers(0, preset.size, size=min(preset.size, 64))
    preset[hot] = rng.integers(0, 2**63, size=hot.size, dtype=np.uint64)
    if nb % 64:  # bits past num_bits stay clear, as a filter's own bits do
        preset[-1] &= np.uint64((1 << (nb % 64)) - 1)
    if offs is None:
        got = ctx.build_fixed(data, key_len, nb, k, words=preset.copy())
        ref = oracle.build_fixed_mt(data, key_len, nb, k, THREADS, words=preset.copy())
    else:
        got = ctx.build_var(data, offs, nb, k, words=preset.copy())
        ref = oracle.build_var_mt(data, offs, nb, k, THREADS, words=preset.copy())
    what = "case %d: %s n=%d num_bits=%d k=%d strategy=%s" % (case, shape, n, nb, k,
                                                             lsmbloom.build_strategy(nb, n, k))
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, "%s: %d words differ, first at %d" % (what, bad.size, bad[0])

    # probe: up to 4000 members and 4000 fresh keys of the same shape
    m = min(n, 4000)
    fdata, foffs, _ = keys_for(rng, shape, 4000, 0x5EED7100 + case)
    if offs is None:
        if key_len != (fdata.size // 4000):  # fixedn: fresh keys of the members' length
            fdata = rng.integers(0, 256, size=4000 * key_len, dtype=np.uint8)
        q = np.concatenate([data[: m * key_len], fdata])
        want = oracle.probe([(ref, nb, k)], q, key_len=key_len)
        ans = ctx.probe([(got, nb, k)], q, key_len=key_len)
    else:
        qd = np.concatenate([data[: int(offs[m])], fdata])
        qo = np.concatenate([offs[: m + 1], foffs[1:] + offs[m]])
        want = oracle.probe([(ref, nb, k)], qd, offsets=qo)
        ans = ctx.probe([(got, nb, k)], qd, offsets=qo)
    assert np.array_equal(ans, want), what
    assert ans[:m, 0].all(), what  # every member hits
