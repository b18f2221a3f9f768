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
controls drop one wait from the schedule and must be caught."""
import random
import threading
import time

import numpy as np
import pytest

from lsmbloom.dist import merge_schedule


class Race(Exception):
    pass


class Sim:
    def __init__(self, world, nwords, seed):
        self.world, self.n = world, nwords
        self.words = [np.zeros(nwords, dtype=np.uint64) for _ in range(world)]
        self.flags = [[0, 0, 0] for _ in range(world)]
        self.lock = threading.Lock()
        self.live = []  # (owner rank of the words, a, b, write, thread rank)
        self.errors = []
        self.rng = random.Random(seed)

    def _enter(self, owner, a, b, write, me):
        with self.lock:
            for (o, x, y, w, t) in self.live:
                if o == owner and t != me and x < b and a < y and (w or write):
                    raise Race("rank %d %s words[%d:%d) of rank %d while rank %d %s [%d:%d)"
                               % (me, "writes" if write else "reads", a, b, owner, t,
                                  "writes" if w else "reads", x, y))
            rec = (owner, a, b, write, me)
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

    def gather(self, me, a, b, srcs, scale):
        recs = [self._enter(r, a, b, False, me) for r in srcs if r != me]
        recs.append(self._enter(me, a, b, True, me))
        try:
            self.pause(scale)
            acc = np.zeros(b - a, dtype=np.uint64)
            for r in srcs:
                acc |= self.words[r][a:b]
                self.pause(scale / 4)
            self.words[me][a:b] = acc
        finally:
            for rec in recs:
                self._leave(rec)

    def wait(self, ph, e, timeout=10.0):
        t0 = time.time()
        while any(self.flags[r][ph] < e for r in range(self.world)):
            if self.errors:  # another rank failed: stop waiting for it
                raise RuntimeError("aborted")
            if time.time() - t0 > timeout:
                raise TimeoutError("phase %d epoch %d never reached" % (ph, e))
            time.sleep(0.0005)


def run(world, nwords, ranges, builds, seed, drop=None, slow_rank=None):
    """Each rank: for each build, rewrite its words with its partial, then merge
    every range in `ranges` (as the overlapped step does per sweep).  Returns
    the snapshots each rank took after each build's last merge."""
    sim = Sim(world, nwords, seed)
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
                            sim.wait(op[1], op[2])
                        elif op[0] == "gather":
                            sim.gather(me, op[1], op[2], op[3], scale)
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
    for bi in range(3):
        want = np.zeros(nwords, dtype=np.uint64)
        for r in range(world):
            want |= partials[bi][r]
        for r in range(world):
            assert np.array_equal(snaps[r][bi], want), (bi, r)


def test_schedule_shape():
    ops = merge_schedule(1, 4, 10, 110, 7)
    kinds = [o[0] for o in ops]
    assert kinds[:2] == ["signal", "wait"] and kinds[-2:] == ["signal", "wait"]
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
