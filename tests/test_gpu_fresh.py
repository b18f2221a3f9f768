"""GPU parity of the fresh-build entry points (lsmb_build_*_dev_new):
BloomFilterBuilder::{new, add_key, build} (src/bloom/builder.rs:14-28) into
OUTPUT-ONLY device words.  The words start as garbage here; every word must
come out equal to the oracle's build into a zeroed filter, for every build
strategy, sweep layout and the overflow (adversarial duplicates) path, whose
side buffer must be left all-zero for the next build.
"""
import numpy as np
import pytest

import keygen
import lsmbloom

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = lsmbloom.Context(0)
    yield c
    c.close()


def _dev():
    import torch
    return torch.device("cuda:0")


def _garbage(nw, seed):
    import torch
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(-2**62, 2**62, (nw,), generator=g, dtype=torch.int64).to(_dev())


def _host(w):
    import torch
    torch.cuda.synchronize()
    return w.cpu().numpy().view(np.uint64)


def _cmp(a, b):
    assert a.shape == b.shape
    bad = np.nonzero(a != b)[0]
    assert bad.size == 0, "first mismatching words: %s" % bad[:8]


@pytest.mark.parametrize("n,filter_keys,fpr,strategy", [
    (50_000, 50_000, 0.01, "lds"),
    (400_000, 1_000_000, 0.01, "tiled"),
    (1000, 10**8, 0.01, "atomic"),
    (4_000_000, 10_000_000, 0.01, "partition"),      # one sweep of 2^20-bit bins
    (8_000_000, 10**9, 0.01, "partition"),           # C5's filter: 2 sweeps of 2^21-bit bins
    (2_000_000, 10**8, 0.001, "partition"),          # k = 10: generic-k kernels
])
def test_fresh_fixed16_on_garbage(ctx, oracle, n, filter_keys, fpr, strategy):
    import torch
    keys_h = keygen.key16(0xF7E5 + n, 0, n)
    nb, k = lsmbloom.params(filter_keys, fpr)
    assert lsmbloom.build_strategy(nb, n, k) == strategy
    keys = torch.from_numpy(keys_h).to(_dev())
    w = _garbage(lsmbloom.num_words(nb), n)
    ctx.build_fixed_dev_new(keys, 16, n, nb, k, w)
    ref = oracle.build_fixed_mt(keys_h, 16, nb, k, 16)
    _cmp(_host(w), ref)


def test_fresh_varlen_and_odd_length_on_garbage(ctx, oracle):
    import torch
    n = 1_000_000
    data, offs = keygen.varlen(n)
    nb, k = lsmbloom.params(10 * n, 0.01)
    assert lsmbloom.build_strategy(nb, n, k) == "partition"
    w = _garbage(lsmbloom.num_words(nb), 7)
    ctx.build_var_dev_new(torch.from_numpy(data).to(_dev()), torch.from_numpy(offs.view(np.int64)).to(_dev()),
                          n, nb, k, w)
    _cmp(_host(w), oracle.build_var_mt(data, offs, nb, k, 16))
    # 24-B keys: the pre-hashed (walk record) pass A
    kl = 24
    raw = keygen.stream_bytes(0x24, n * kl)
    w = _garbage(lsmbloom.num_words(nb), 8)
    ctx.build_fixed_dev_new(torch.from_numpy(raw).to(_dev()), kl, n, nb, k, w)
    _cmp(_host(w), oracle.build_fixed_mt(raw, kl, nb, k, 16))


@pytest.mark.parametrize("filter_keys", [10_000_000, 10**9])
def test_fresh_overflow_side_buffer(ctx, oracle, filter_keys):
    """Duplicate-heavy keys overflow rings and regions: those positions go to
    the overflow words (never to the output words, which a fresh build does
    not read) and pass B folds them in.  2^20-bit bins (one sweep) and the
    2^21-bit bins of C5's 2-sweep filter.  The overflow words must be all-zero
    again afterwards: an accumulate build with overflow and a clean fresh
    build follow on the same context."""
    import torch
    n = 10_000_000
    keys_h = keygen.key16(0xD00D, 0, n)
    keys_h[:2_000_000] = keys_h[0]
    keys_h[2_000_000:3_000_000] = keys_h[5_000_000]
    nb, k = lsmbloom.params(filter_keys, 0.01)
    keys = torch.from_numpy(keys_h).to(_dev())
    w = _garbage(lsmbloom.num_words(nb), 11)
    ctx.build_fixed_dev_new(keys, 16, n, nb, k, w)
    ref = oracle.build_fixed_mt(keys_h, 16, nb, k, 16)
    _cmp(_host(w), ref)
    # accumulate mode on top of a preset: overflow bits OR into the old words
    pre = np.zeros(lsmbloom.num_words(nb), np.uint64)
    pre[::101] = 0x8000000000000001
    w2 = torch.from_numpy(pre.view(np.int64)).to(_dev())
    ctx.build_fixed_dev(keys, 16, n, nb, k, w2)
    _cmp(_host(w2), ref | pre)
    # a clean build afterwards sees no stale overflow bits
    clean_h = keygen.key16(0xC1EA, 0, 1_000_000)
    w3 = _garbage(lsmbloom.num_words(nb), 12)
    ctx.build_fixed_dev_new(torch.from_numpy(clean_h).to(_dev()), 16, 1_000_000, nb, k, w3)
    _cmp(_host(w3), oracle.build_fixed_mt(clean_h, 16, nb, k, 16))


def test_fresh_sweeps_write_their_range_only(ctx, oracle):
    import torch
    n = 6_000_000
    keys_h = keygen.key16(0x5EE9, 0, n)
    nb, k = lsmbloom.params(10**9, 0.01)
    ns = lsmbloom.build_sweeps(nb, n, k)
    assert ns == 2
    keys = torch.from_numpy(keys_h).to(_dev())
    w = _garbage(lsmbloom.num_words(nb), 21)
    before = _host(w).copy()
    ref = oracle.build_fixed_mt(keys_h, 16, nb, k, 16)
    lo, hi = lsmbloom.sweep_words(nb, n, 0, k)
    ctx.build_fixed_dev_sweep_new(keys, 16, n, nb, k, w, 0)
    got = _host(w)
    _cmp(got[lo:hi], ref[lo:hi])
    _cmp(got[hi:], before[hi:])  # the other sweep's words untouched
    ctx.build_fixed_dev_sweep_new(keys, 16, n, nb, k, w, 1)
    _cmp(_host(w), ref)


def test_fresh_empty_and_k0(ctx):
    import torch
    nb, k = lsmbloom.params(10**8, 0.01)
    w = _garbage(lsmbloom.num_words(nb), 31)
    ctx.build_fixed_dev_new(torch.empty(0, dtype=torch.uint8, device=_dev()), 16, 0, nb, k, w)
    assert not _host(w).any()  # new() with no inserts
    w = _garbage(lsmbloom.num_words(nb), 32)
    keys = torch.from_numpy(keygen.key16(1, 0, 1000)).to(_dev())
    ctx.build_fixed_dev_new(keys, 16, 1000, nb, 0, w)
    assert not _host(w).any()  # k = 0: insert sets nothing


def test_c2_fresh_full_size_fixture(ctx):
    """C2 (100 M key16 into new(1e8, 0.01)) through the fresh entry point, into
    words that start as all-ones: every word against the oracle's digest."""
    import torch
    from test_gpu_parity import assert_full_fixture
    n = 100_000_000
    nb, k = lsmbloom.params(n, 0.01)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=_dev())
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    w = torch.full((lsmbloom.num_words(nb),), -1, dtype=torch.int64, device=_dev())
    ctx.build_fixed_dev_new(keys, 16, n, nb, k, w)
    assert_full_fixture(_host(w), "c2")
