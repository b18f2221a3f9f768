"""C3 (BASELINE configs[2]) at full size on the host: the workload bench.py's
probe leg builds on the device, and the oracle's answers for it.  TEST
INFRASTRUCTURE: tests/golden/gen_c3_fixture.py writes the answers' digests
(tests/golden/c3_fixture.json) that bench.py compares with, and
tests/test_gpu_parity.py compares every answer byte with these arrays.

Workload (bench.py bench_probe): F = 8 SSTable filters sized like
SSTableBuilder::new (new(1000, 0.01): 9 568 bits, k = 7,
src/sstable/builder.rs:51,74), filter f built from key16(0xF000 + f, 0..1000);
Q = 10 M lookup keys key16(0x5EED0002, 0..Q) whose first Q/2 rows are replaced
by member rows drawn with torch.randint(0, 8000, (Q/2,), Generator seed 1).
Answers: may_contain per (key, filter) — src/sstable/reader.rs:197 — as one
mask byte per key; and the filter-set form (lsmb_fset), which also applies
SSTable::get's range pre-check min_key <= key <= max_key (reader.rs:192-194)
with each table's range = its members' min / max rows.
"""
import hashlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

SEED_FRESH = 0x5EED0002


def workload(orc, Q=10_000_000, F=8):
    import torch
    members = np.concatenate([orc.key16(0xF000 + f, 0, 1000) for f in range(F)])
    q = orc.key16(SEED_FRESH, 0, Q)
    g = torch.Generator(device="cpu").manual_seed(1)
    sel = torch.randint(0, F * 1000, (Q // 2,), generator=g).numpy()
    q[: Q // 2] = members[sel]
    return members, q, sel


def _be2(rows):
    """16-B rows -> (hi, lo) big-endian u64 pairs: their order is the rows' byte order."""
    r = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, 16)
    return r[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64), r[:, 8:].copy().view(">u8").reshape(-1).astype(np.uint64)


def in_range(q, lo_row, hi_row):
    qh, ql = _be2(q)
    (lh,), (ll,) = _be2(lo_row)
    (hh,), (hl,) = _be2(hi_row)
    ge = (qh > lh) | ((qh == lh) & (ql >= ll))
    le = (qh < hh) | ((qh == hh) & (ql <= hl))
    return ge & le


def probe_mt(orc, filters, q, threads=8):
    parts = np.array_split(np.arange(q.shape[0]), threads)
    with ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(lambda ix: orc.probe(filters, q[ix[0]:ix[-1] + 1], key_len=16) if ix.size else
                           np.zeros((0, (len(filters) + 7) // 8), np.uint8), parts))
    return np.concatenate(outs)


def sorted_bounds(rows):
    srt = sorted(bytes(r) for r in rows)
    return np.frombuffer(srt[0], np.uint8), np.frombuffer(srt[-1], np.uint8)


def answers(orc, Q=10_000_000, F=8, threads=8):
    """(probe mask bytes [Q, ceil(F/8)], fset u64 masks [Q], mixed-set u64 masks [Q])."""
    members, q, _ = workload(orc, Q, F)
    nb, k = orc.params(1000, 0.01)
    filt = [(orc.build_fixed(members[f * 1000:(f + 1) * 1000], 16, nb, k), nb, k) for f in range(F)]
    mask = probe_mt(orc, filt, q, threads)
    fset = np.zeros(Q, np.uint64)
    for f in range(F):
        lo, hi = sorted_bounds(members[f * 1000:(f + 1) * 1000])
        hit = ((mask[:, f // 8] >> (f % 8)) & 1).astype(bool)
        fset |= (hit & in_range(q, lo, hi)).astype(np.uint64) << np.uint64(f)
    # mixed sizes: 4 C3 tables + 4 compaction-sized new(4000, 0.01) tables
    nb4, k4 = orc.params(4000, 0.01)
    mixed = np.zeros(Q, np.uint64)
    for f in range(F):
        if f < F // 2:
            rows, fl = members[f * 1000:(f + 1) * 1000], filt[f]
        else:
            rows = orc.key16(0xF100 + f, 0, 4000)
            fl = (orc.build_fixed(rows, 16, nb4, k4), nb4, k4)
        hit = probe_mt(orc, [fl], q, threads)[:, 0].astype(bool)
        lo, hi = sorted_bounds(rows)
        mixed |= (hit & in_range(q, lo, hi)).astype(np.uint64) << np.uint64(f)
    return mask, fset, mixed


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
