"""Host model of k_bin_pk's packed-ring fill word (csrc/bloom_build.hip,
"packed-ring pass A"): the slot / field a claim gets back from its
ds_add_rtn, for every flush state and every claim count up to the ring.

Fill word: bits 0-12 fraction of a slot, 13-17 slot (mod 32), 18-31 claims;
a claim adds 1 << 18 | 2731.  A claim's ring byte offset is
(fill >> 10) & 0x78 and its field shift (fill >> 7) mod 64.
"""
import pytest

INC = (1 << 18) | 2731
SLOTS, ENTRIES, FIELD = 16, 48, 21
SEG = 24


def frac(r):
    return (0, 2731, 5462)[r]


def owner_rewrite(start, rem):
    # the owner's fill after a flush: start (bytes, 0 or 64), rem entries left
    return frac(rem % 3) | (((start >> 3) + rem // 3) << 13) | (rem << 18)


def claims(fill, c):
    out = []
    for _ in range(c):
        out.append(fill)
        fill = (fill + INC) & 0xFFFFFFFF
    return out, fill


@pytest.mark.parametrize("start", [0, 64])
def test_claims_fill_the_ring_in_order(start):
    lim = ENTRIES << 18
    for rem in range(SEG):
        f0 = owner_rewrite(start, rem)
        got, _ = claims(f0, ENTRIES - rem + 5)
        seen = set()
        for i, g in enumerate(got):
            e = rem + i  # entry index from the ring start
            if e >= ENTRIES:
                assert g >= lim  # past the ring: the overflow path
                continue
            assert g < lim
            off = (g >> 10) & ((SLOTS - 1) * 8)
            sh = (g >> 7) & 63
            want_slot = ((start >> 3) + e // 3) % SLOTS
            assert off == 8 * want_slot, (start, rem, i)
            assert sh == FIELD * (e % 3), (start, rem, i)
            assert (off, sh) not in seen
            seen.add((off, sh))


def test_phase_claims_never_reach_the_count():
    # the slot field (5 bits) holds start + claims / 3 for every in-ring claim
    for start in (0, 64):
        for rem in range(SEG):
            got, _ = claims(owner_rewrite(start, rem), ENTRIES - rem)
            for g in got:
                assert (g >> 18) < ENTRIES


def test_adversarial_counts_stay_monotone():
    # 2048 keys x 7 positions into one bin in one phase: the count never wraps
    got, last = claims(owner_rewrite(64, 23), 2048 * 7)
    counts = [g >> 18 for g in got]
    assert all(b >= a for a, b in zip(counts, counts[1:]))
    assert counts[ENTRIES - 23] >= ENTRIES
    assert last >> 18 < (1 << 14)
