"""The device-ordered IPC merge protocol (lsmbloom.dist.merge_schedule) run
against simulated ranks on the CPU: one thread per rank
plays its stream in order — builds that rewrite all of its words, then the
merge's signal / wait / gather ops — over shared word arrays and flag arrays.
Every access to a rank's words is registered with its word range; a write that
overlaps another thread's live access to the same words (or a read that
overlaps a live write) is a race.  Random delays widen every window.

Checked: no race, and after each merge every rank holds the OR of all ranks'
partials of that build, across consecutive builds (the overlapped N > 1 step
of bench.py, which rebuilds the words right after a merge).  The negative
controls drop one wait from the schedule and must be caught.  run_streams plays
the overlapped and pipelined step forms with two streams per rank (a build
stream rewriting one sweep's range while the side stream merges another).

The fail-safe: with a short timeout, a rank that dies
after its build, or stalls past the timeout, must never make a live rank end
a merge with a bit of the true OR missing; a rank whose words are not the
exact OR must have its poison set (the error its host raises)."""
import random
import threading
import time

import numpy as np
import pytest

from lsmbloom.dist import merge_schedule


ONES = np.uint64(2 ** 64 - 1)


class Race(Exception):
    pass


class Sim:
    """Shared state of the simulated ranks.  strict=True (the protocol tests):
    any overlap of a write with another thread's live access to the same words
    raises Race.  strict=False (the fail-safe tests, where a rank that gave up
    on a dead or stalled peer may rewrite words a slow peer still reads): the
    overlapping read is torn instead, and a torn read contributes no bits at
    all — the worst case for a Bloom filter, a false negative."""

    def __init__(self, world, nwords, seed, strict=True, timeout=10.0):
        self.world, self.n, self.strict, self.timeout = world, nwords, strict, timeout
        self.words = [np.zeros(nwords, dtype=np.uint64) for _ in range(world)]
        self.flags = [[0, 0, 0] for _ in range(world)]
        self.poison = [0] * world    # status word [0], read by every rank's waits
        self.timeouts = [0] * world  # status word [1]
        self.lock = threading.Lock()
        self.live = []  # [owner rank of the words, a, b, write, thread rank, torn]
        self.errors = []
        self.rng = random.Random(seed)

    def _enter(self, owner, a, b, write, me):
        with self.lock:
            rec = [owner, a, b, write, me, False]
            for other in self.live:
                o, x, y, w, t, _ = other
                if o == owner and t != me and x < b and a < y and (w or write):
                    if self.strict:
                        raise Race("rank %d %s words[%d:%d) of rank %d while rank %d %s [%d:%d)"
                                   % (me, "writes" if write else "reads", a, b, owner, t,
                                      "writes" if w else "reads", x, y))
                    if write:
                        other[5] = True  # the other thread's read is torn
                    else:
                        rec[5] = True
            self.live.append(rec)
            return rec

    def _leave(self, rec):
        with self.lock:
            self.live.remove(rec)

    def pause(self, scale):
        time.sleep(self.rng.random() * scale)

    def build(self, me, partial, scale):
        rec = self._enter(me, 0, self.n, True, me)
        try:
            self.pause(scale)
            self.words[me][:] = partial
            self.pause(scale)
        finally:
            self._leave(rec)

    def fill(self, me, a, b, scale):
        rec = self._enter(me, a, b, True, me)
        try:
            self.pause(scale / 4)
            self.words[me][a:b] = ONES
        finally:
            self._leave(rec)

    def gather(self, me, a, b, srcs, scale):
        """k_or_gather / one slice of k_copy_slices: my words[a:b] = OR of the
        sources' words[a:b]; poisoned, all-ones and no source read."""
        if self.poison[me]:
            self.fill(me, a, b, scale)
            return
        recs = {r: self._enter(r, a, b, False, me) for r in srcs if r != me}
        mine = self._enter(me, a, b, True, me)
        try:
            self.pause(scale)
            acc = np.zeros(b - a, dtype=np.uint64)
            for r in srcs:
                if r in recs and recs[r][5]:
                    continue  # torn: no bits
                acc |= self.words[r][a:b]
                self.pause(scale / 4)
            self.words[me][a:b] = acc
        finally:
            for rec in list(recs.values()) + [mine]:
                self._leave(rec)

    def wait(self, me, ph, e):
        """k_flag_wait: until every flags[ph] >= e; any rank's poison (mine
        included) ends it and poisons me; so does a timeout (counted); every
        poison word is read once more after the flags were met."""
        t0 = time.time()
        while any(self.flags[r][ph] < e for r in range(self.world)):
            if self.errors:  # another rank failed: stop waiting for it
                raise RuntimeError("aborted")
            if any(self.poison):
                break
            if time.time() - t0 > self.timeout:
                if self.strict:
                    raise TimeoutError("phase %d epoch %d never reached" % (ph, e))
                self.timeouts[me] += 1
                self.poison[me] = 1
                return
            time.sleep(0.0005)
        if any(self.poison):
            self.poison[me] = 1


def run(world, nwords, ranges, builds, seed, drop=None, slow_rank=None, strict=True, timeout=10.0,
        dead_rank=None, stall=None):
    """Each rank: for each build, rewrite its words with its partial, then merge
    every range in `ranges` (as the overlapped step does per sweep).  Returns
    the snapshots each rank took after each build's last merge.  dead_rank:
    that rank builds once and stops (never signals).  stall = (rank, build,
    seconds): that rank sleeps before the build's merges (alive, but late)."""
    sim = Sim(world, nwords, seed, strict=strict, timeout=timeout)
    rng = np.random.default_rng(seed)
    partials = [[rng.integers(0, 2 ** 63, nwords, dtype=np.uint64) & rng.integers(0, 2 ** 63, nwords, dtype=np.uint64)
                 for _ in range(world)] for _ in range(builds)]
    snaps = [[None] * builds for _ in range(world)]

    def rank_main(me):
        try:
            epoch = 0
            for bi in range(builds):
                scale = 0.004 if me == slow_rank else 0.0015
                sim.build(me, partials[bi][me], scale)
                if me == dead_rank:
                    return
                if stall and stall[:2] == (me, bi):
                    time.sleep(stall[2])
                for (lo, hi) in ranges:
                    epoch += 1
                    for op in merge_schedule(me, world, lo, hi, epoch):
                        if drop and op[:2] == drop:
                            continue
                        if op[0] == "signal":
                            sim.pause(scale / 2)
                            with sim.lock:
                                sim.flags[me][op[1]] = op[2]
                        elif op[0] == "wait":
                            sim.wait(me, op[1], op[2])
                        elif op[0] == "gather":
                            sim.gather(me, op[1], op[2], op[3], scale)
                        elif op[0] == "fill":
                            if sim.poison[me]:
                                sim.fill(me, op[1], op[2], scale)
                        else:  # copy: each listed rank's slice of [lo, hi) from that rank
                            _, lo, hi, per, srcs = op
                            for r in srcs:
                                sim.gather(me, min(hi, lo + r * per), min(hi, lo + (r + 1) * per), [r], scale)
                snaps[me][bi] = sim.words[me].copy()
        except Exception as ex:  # reported by the main thread
            sim.errors.append(ex)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    return sim, partials, snaps


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_device_ordered_merge_has_no_race_and_merges(world):
    nwords = 64 * world + 6
    ranges = [(0, nwords // 2), (nwords // 2, nwords)]  # two sweeps' word ranges
    sim, partials, snaps = run(world, nwords, ranges, builds=3, seed=world)
    assert not sim.errors, sim.errors[0]
    assert not any(sim.poison) and not any(sim.timeouts)
    for bi in range(3):
        want = np.zeros(nwords, dtype=np.uint64)
        for r in range(world):
            want |= partials[bi][r]
        for r in range(world):
            assert np.array_equal(snaps[r][bi], want), (bi, r)


def test_schedule_shape():
    ops = merge_schedule(1, 4, 10, 110, 7)
    kinds = [o[0] for o in ops]
    assert kinds[:2] == ["signal", "wait"] and kinds[-3:] == ["signal", "wait", "fill"]
    assert ops[-1] == ("fill", 10, 110)  # a poisoned merge ends with its whole range all-ones
    assert [o[1] for o in ops if o[0] == "signal"] == [0, 1, 2]
    g = [o for o in ops if o[0] == "gather"]
    assert g == [("gather", 36, 62, [0, 1, 2, 3])]  # my slice (per = 26), all ranks' partials
    c = [o for o in ops if o[0] == "copy"]
    assert c == [("copy", 10, 110, 26, [0, 2, 3])]  # every other rank's slice, one kernel
    assert kinds.index("gather") < kinds.index("copy")
    assert all(o[2] == 7 for o in ops if o[0] in ("signal", "wait"))
    # ragged: the last slice is short or empty; a rank whose slice is empty copies only
    ops = merge_schedule(3, 4, 0, 6, 1)
    assert [o for o in ops if o[0] == "gather"] == []
    assert [o[0] for o in merge_schedule(0, 2, 5, 5, 1)][-1] == "wait"  # empty range: nothing to fill
    assert [o for o in ops if o[0] == "copy"] == [("copy", 0, 6, 2, [0, 1, 2])]


@pytest.mark.parametrize("drop,slow", [(("wait", 2), 1), (("wait", 0), 0), (("wait", 1), 2)])
def test_dropping_a_wait_is_caught(drop, slow):
    """Negative controls: without the last wait a fast rank rebuilds its words
    while a slow peer still copies from them; without the first, a gather reads
    a peer mid-build; without the middle one, a copy reads a slice that is still
    being merged.  The checker must see a race or a wrong merge."""
    world, nwords = 3, 3 * 64
    caught = 0
    for seed in range(12):
        sim, partials, snaps = run(world, nwords, [(0, nwords)], builds=3, seed=100 + seed, drop=drop,
                                   slow_rank=slow)
        if sim.errors:
            caught += 1
            continue
        for bi in range(3):
            want = np.zeros(nwords, dtype=np.uint64)
            for r in range(world):
                want |= partials[bi][r]
            if any(snaps[r][bi] is None or not np.array_equal(snaps[r][bi], want) for r in range(world)):
                caught += 1
                break
    assert caught > 0


def _want(partials, bi, world):
    want = np.zeros(partials[bi][0].size, dtype=np.uint64)
    for r in range(world):
        want |= partials[bi][r]
    return want


@pytest.mark.parametrize("world,dead", [(2, 1), (3, 0), (4, 2), (8, 5)])
def test_dead_rank_leaves_live_ranges_all_ones(world, dead):
    """a rank that dies after its build never signals.
    Every live rank's waits time out or see a peer's poison: its merged ranges
    end all-ones (a superset of the true OR: no false negative), its poison is
    set, and at least one live rank counted a timeout — the error the host
    raises at its next sync point (IpcMerge.check / allreduce(check=True))."""
    nwords = 16 * world + 6
    ranges = [(0, nwords // 2), (nwords // 2, nwords)]
    sim, partials, snaps = run(world, nwords, ranges, builds=2, seed=7 + world, strict=False, timeout=0.05,
                               dead_rank=dead)
    assert not sim.errors, sim.errors[0]
    live = [r for r in range(world) if r != dead]
    for r in live:
        assert sim.poison[r], r
        for bi in range(2):
            assert snaps[r][bi] is not None and (snaps[r][bi] == ONES).all(), (r, bi)
    assert sum(sim.timeouts[r] for r in live) >= 1


@pytest.mark.parametrize("seed", range(6))
def test_stalled_rank_never_yields_missing_bits(seed):
    """A rank that is alive but stalls past the timeout before a build's merges:
    the others give up on it, poison, and go on to rebuild their words while it
    may still read them (reads that overlap a rewrite are torn and lose their
    bits here).  Whatever the interleaving, no rank ever ends a merge with a
    bit of the true OR missing, and every rank whose words are not the exact
    OR has its poison set."""
    world, nwords = 3, 3 * 32
    ranges = [(0, nwords // 2), (nwords // 2, nwords)]
    stall = (seed % world, 1, 0.25)
    sim, partials, snaps = run(world, nwords, ranges, builds=3, seed=300 + seed, strict=False, timeout=0.05,
                               stall=stall)
    assert not sim.errors, sim.errors[0]
    assert any(sim.poison)
    for bi in range(3):
        want = _want(partials, bi, world)
        for r in range(world):
            got = snaps[r][bi]
            assert got is not None
            assert ((got & want) == want).all(), "rank %d build %d lost bits" % (r, bi)
            if not np.array_equal(got, want):
                assert sim.poison[r], "rank %d build %d inexact but not poisoned" % (r, bi)


def test_failsafe_checker_catches_a_missing_poison_check():
    """Negative control for the fail-safe tests: with poison ignored by the
    gathers (a rank that gave up still reads and OR-merges, and nobody writes
    all-ones), a dead peer leaves live ranks with bits missing."""
    world, nwords = 3, 3 * 16
    orig = Sim.gather

    def careless(self, me, a, b, srcs, scale):
        p, self.poison[me] = self.poison[me], 0
        try:
            return orig(self, me, a, b, srcs, scale)
        finally:
            self.poison[me] = p
    Sim.gather = careless
    try:
        sim, partials, snaps = run(world, nwords, [(0, nwords)], builds=1, seed=5, strict=False, timeout=0.05,
                                   dead_rank=2)
    finally:
        Sim.gather = orig
    # the fill still runs, so a careless gather alone is masked by it...
    assert all((snaps[r][0] == ONES).all() for r in (0, 1))
    # ...and without the fill too, bits go missing
    orig_fill = Sim.fill
    Sim.gather, Sim.fill = careless, lambda self, me, a, b, scale: None
    try:
        _, partials, snaps = run(world, nwords, [(0, nwords)], builds=1, seed=5, strict=False, timeout=0.05,
                                    dead_rank=2)
    finally:
        Sim.gather, Sim.fill = orig, orig_fill
    want = _want(partials, 0, world)
    assert any(not ((snaps[r][0] & want) == want).all() for r in (0, 1))


def _build_range(sim, me, values, lo, hi, scale):
    """A fresh sweep: rewrites my words[lo:hi] (its own range and nothing else)."""
    rec = sim._enter(me, lo, hi, True, me)
    try:
        sim.pause(scale)
        sim.words[me][lo:hi] = values
        sim.pause(scale)
    finally:
        sim._leave(rec)


def run_streams(world, nwords, ranges, builds, seed, form, skip_merge_wait=False):
    """bench.py's N > 1 step forms with two streams per rank, one thread each:
    the build stream runs sweep s of build b (rewriting range s only), the
    side stream merges range s once that sweep is done (merge_schedule, epochs
    in merge order).  Before sweep s of build b+1 the build stream waits for
    range s's merge of build b ("pipelined") or for every merge of build b
    ("overlapped": the step ends with the side stream).  Each merge snapshots
    its range before it releases the build stream.  skip_merge_wait: the build
    stream waits for nothing (the negative control)."""
    sim = Sim(world, nwords, seed)
    rng = np.random.default_rng(seed)
    partials = [[rng.integers(0, 2 ** 63, nwords, dtype=np.uint64) & rng.integers(0, 2 ** 63, nwords, dtype=np.uint64)
                 for _ in range(world)] for _ in range(builds)]
    snaps = [[np.zeros(nwords, dtype=np.uint64) for _ in range(builds)] for _ in range(world)]

    def rank_main(me):
        built = [[threading.Event() for _ in ranges] for _ in range(builds)]
        merged = [[threading.Event() for _ in ranges] for _ in range(builds)]
        scale = 0.0015

        def need(ev):
            t0 = time.time()
            while not ev.wait(0.01):
                if sim.errors:  # another stream failed: stop waiting for it
                    raise RuntimeError("aborted")
                if time.time() - t0 > 20:
                    raise TimeoutError("stream event never set")

        def main():
            try:
                for bi in range(builds):
                    for s, (lo, hi) in enumerate(ranges):
                        if bi and not skip_merge_wait:
                            for t in ([s] if form == "pipelined" else range(len(ranges))):
                                need(merged[bi - 1][t])
                        _build_range(sim, me, partials[bi][me][lo:hi], lo, hi, scale)
                        built[bi][s].set()
            except Exception as ex:
                sim.errors.append(ex)

        def side():
            try:
                epoch = 0
                for bi in range(builds):
                    for s, (lo, hi) in enumerate(ranges):
                        need(built[bi][s])
                        epoch += 1
                        for op in merge_schedule(me, world, lo, hi, epoch):
                            if op[0] == "signal":
                                sim.pause(scale / 2)
                                with sim.lock:
                                    sim.flags[me][op[1]] = op[2]
                            elif op[0] == "wait":
                                sim.wait(me, op[1], op[2])
                            elif op[0] == "gather":
                                sim.gather(me, op[1], op[2], op[3], scale)
                            elif op[0] == "fill":
                                if sim.poison[me]:
                                    sim.fill(me, op[1], op[2], scale)
                            else:
                                _, a, b, per, srcs = op
                                for r in srcs:
                                    sim.gather(me, min(b, a + r * per), min(b, a + (r + 1) * per), [r], scale)
                        snaps[me][bi][lo:hi] = sim.words[me][lo:hi]
                        merged[bi][s].set()
            except Exception as ex:
                sim.errors.append(ex)

        th = [threading.Thread(target=main), threading.Thread(target=side)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(90)
    return sim, partials, snaps


@pytest.mark.parametrize("world,form", [(2, "pipelined"), (3, "pipelined"), (4, "pipelined"), (3, "overlapped")])
def test_step_forms_with_two_streams_have_no_race(world, form):
    """The overlapped and pipelined N > 1 steps (bench.py): sweep s of the next
    build rewrites range s while other ranges still merge on the side stream.
    No race, and every merge leaves every rank with the exact OR of that
    build's partials over its range."""
    nwords = 32 * world + 6
    ranges = [(0, nwords // 2), (nwords // 2, nwords)]
    sim, partials, snaps = run_streams(world, nwords, ranges, builds=4, seed=40 + world, form=form)
    assert not sim.errors, sim.errors[0]
    assert not any(sim.poison) and not any(sim.timeouts)
    for bi in range(4):
        want = _want(partials, bi, world)
        for r in range(world):
            assert np.array_equal(snaps[r][bi], want), (form, bi, r)


def test_step_forms_checker_catches_a_build_that_skips_the_merge_event():
    """Negative control: a build stream that starts sweep s of the next build
    without waiting for range s's merge rewrites words a peer may still read."""
    world, nwords = 3, 3 * 32
    ranges = [(0, nwords // 2), (nwords // 2, nwords)]
    caught = 0
    for seed in range(8):
        sim, partials, snaps = run_streams(world, nwords, ranges, builds=3, seed=500 + seed, form="pipelined",
                                           skip_merge_wait=True)
        if sim.errors or any(not np.array_equal(snaps[r][bi], _want(partials, bi, world))
                             for bi in range(3) for r in range(world)):
            caught += 1
    assert caught > 0
