"""Multi-GPU: merge per-rank partial filters with a bitwise-OR allreduce.

A sharded build (each rank hashes its contiguous slice of one run's keys into
a full-size partial filter) is exact because OR is associative, commutative and
idempotent: OR of the partials == the single-device filter, bit for bit.

RCCL has no bitwise-OR reduction (rccl.h ncclRedOp_t: sum/prod/max/min/avg),
so the allreduce is composed from op-free collectives:
  1. reduce-scatter: all_to_all_single sends word-slice j of my partial to rank j;
  2. each rank ORs the G slices it received (native kernel, lsmb_or_reduce_dev);
  3. all_gather_into_tensor returns the merged slices to every rank.
Per-GPU traffic is 2 (G-1)/G x filter bytes; over xGMI's point-to-point links
the all_to_all phase uses every peer link at once.  The end-to-end variant
(`or_reduce_scatter_`) stops after step 2: each rank then copies its own slice
to host memory, which parallelises the D2H over the ranks' PCIe links.
"""
import torch
import torch.distributed as dist


def _slices(n, world):
    per = (n + world - 1) // world
    per = (per + 1) & ~1  # even: 16-B aligned slices of int64 words
    return per


def _host_staged(words, group):
    """gloo moves host memory only: device words are staged through it (the
    one-GPU multi-rank tests); RCCL (nccl) works on device memory directly."""
    return words.is_cuda and dist.get_backend(group) == "gloo"


def or_reduce_scatter_(words, group=None, ctx=None):
    """Returns (slice_tensor, start_word): this rank's merged slice of the filter."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = words.numel()
    per = _slices(n, world)
    if per * world != n:
        buf = torch.zeros(per * world, dtype=words.dtype, device=words.device)
        buf[:n].copy_(words)
    else:
        buf = words
    if _host_staged(words, group):
        recv_h = torch.empty(buf.shape, dtype=buf.dtype)
        dist.all_to_all_single(recv_h, buf.cpu(), group=group)
        recv = recv_h.to(words.device)
    else:
        recv = torch.empty_like(buf)
        dist.all_to_all_single(recv, buf, group=group)
    mine = torch.empty(per, dtype=words.dtype, device=words.device)
    if words.is_cuda and ctx is not None:
        mine.zero_()
        ctx.or_reduce_dev(mine, recv, per, world, per)
    else:
        r = recv.view(world, per)
        mine.copy_(r[0])
        for j in range(1, world):
            mine.bitwise_or_(r[j])
    return mine, rank * per


def or_allreduce_(words, group=None, ctx=None):
    """In-place bitwise-OR allreduce of an int64 word tensor across the group."""
    world = dist.get_world_size(group)
    if world == 1:
        return words
    n = words.numel()
    mine, _ = or_reduce_scatter_(words, group, ctx)
    per = mine.numel()
    if _host_staged(words, group):
        out = torch.empty(per * world, dtype=words.dtype)
        dist.all_gather_into_tensor(out, mine.cpu(), group=group)
        words.copy_(out[:n])
        return words
    if per * world == n and words.is_contiguous():
        dist.all_gather_into_tensor(words, mine, group=group)  # no staging copy (C5: 2^26 words)
        return words
    out = torch.empty(per * world, dtype=words.dtype, device=words.device)
    dist.all_gather_into_tensor(out, mine, group=group)
    words.copy_(out[:n])
    return words


class MergePoisoned(RuntimeError):
    """An IpcMerge whose phase waits timed out (a peer died or stalled past
    timeout_ms) or that saw another rank's poison.  Its ranges were written
    all-ones from that point on, so the filter has no false negatives, but it
    is not the exact merge: do not serialize it as the run's filter."""


# A rank's flag array (device int32, exported to the peers): the three phase
# epochs, then the merge's status words (include/lsmbloom.h,
# LSMB_MERGE_STATUS_WORDS): poison (published to the peers) and timed-out waits.
_PHASES = 3
_POISON = 3
_TIMEOUTS = 4
_FLAG_WORDS = 8


class IpcMerge:
    """The OR-allreduce by peer loads between processes (one per GPU), with no
    collective library on the data path (include/lsmbloom.h, "cross-process
    peer-load merge"): every rank exports the device allocation holding its
    words once, maps every other rank's (lsmb_ipc_import: xGMI peer mappings
    across GPUs, the same HBM when ranks share one), and merges a word range
    in two peer-load kernels:
      1. reduce-scatter: rank g ORs word-slice g of all G partials into its own
         words (one lsmb_or_gather_dev, G sources);
      2. all-gather: rank g copies every other merged slice from its owner.
    Per GPU it reads (G-1)/G of the range twice over the peer links, the RCCL
    path's bytes.

    Ordering.  ordered="host" (the default): a stream synchronise plus a
    `group` barrier between phases.  ordered="device": the phases are ordered
    on the GPUs, never on the host.  Every rank also exports a flag array;
    merge number e enqueues on the caller's stream
        signal(my flag[0] = e); wait(every rank's flag[0] >= e)   partials final
        reduce-scatter;  signal(flag[1] = e); wait(all flag[1] >= e)
        all-gather;      signal(flag[2] = e); wait(all flag[2] >= e)
        poison fill
    (lsmb_flag_signal_dev / lsmb_flag_wait_dev) and returns at once: the host
    never synchronises inside a merge, so a sweep's merge overlaps the next
    sweep's build.  The last wait keeps any later work on the stream from
    rewriting my words while a peer may still read them.  `merge_schedule`
    below is the protocol as data (tests/test_ipc_protocol.py runs it against
    simulated ranks).  The device-ordered form has run with every rank on one
    GPU only; bench.py selects it explicitly, after checking its words against
    RCCL's on the node it runs on.

    Fail-safe (device-ordered).  A wait that times out (a dead or stalled
    peer), or that sees another rank's poison word, poisons this merge for
    good: from then on its kernels read no peer words and write all-ones, and
    the merge's range ends all-ones — a superset of every partial, so the
    filter may answer "maybe" too often but never "no" for an added key.  The
    error surfaces at the next sync point: allreduce(..., check=True),
    check(), or close().

    `group` (gloo) exchanges the handles once, checks each new word range once
    against every rank's, and orders close()."""

    def __init__(self, words, ctx, group=None, ordered="host", timeout_ms=20000):
        import lsmbloom
        if ordered not in ("device", "host"):
            raise ValueError("ordered must be 'device' or 'host'")
        self.words, self.ctx, self.group, self.ordered = words, ctx, group, ordered
        self.timeout_ms = int(timeout_ms)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.epoch = 0
        self._checked = set()
        # phase flags (epochs) and status words, zero before any peer can poll
        # them: the handle exchange below happens after this synchronise
        self.flags = torch.zeros(_FLAG_WORDS, dtype=torch.int32, device=words.device)
        torch.cuda.synchronize(words.device)
        h, off = lsmbloom.ipc_export(words)
        fh, foff = lsmbloom.ipc_export(self.flags)
        allh = [None] * self.world
        dist.all_gather_object(allh, (h, off, words.numel(), fh, foff), group=group)
        self.bases, self.ptrs, self.fptrs = [], [], []
        for r, (hh, oo, n, fhh, foo) in enumerate(allh):
            if n != words.numel():
                raise ValueError("rank %d's words hold %d words, mine %d" % (r, n, words.numel()))
            if r == self.rank:
                self.ptrs.append(words.data_ptr())
                self.fptrs.append(self.flags.data_ptr())
                continue
            base = ctx.ipc_import(hh)
            self.bases.append(base)
            self.ptrs.append(base + oo)
            if fhh == hh:  # the flags share the words' allocation: one mapping
                self.fptrs.append(base + foo)
            else:
                fbase = ctx.ipc_import(fhh)
                self.bases.append(fbase)
                self.fptrs.append(fbase + foo)
        self.status_ptr = self.fptrs[self.rank] + 4 * _POISON

    def status(self, stream=None):
        """(poisoned, timed-out waits) of this merge so far, after `stream`'s
        pending work (default: the current stream; synchronises it)."""
        stream = stream or torch.cuda.current_stream(self.words.device)
        p, t = self.ctx.merge_status(self.status_ptr, stream=stream.cuda_stream)
        return bool(p), t

    def timeouts(self, stream=None):
        """Phase waits of this merge that timed out so far."""
        return self.status(stream)[1]

    def check(self, stream=None):
        """The merge's sync point: raises MergePoisoned if any merge so far was
        poisoned (its ranges are all-ones, not the exact OR)."""
        p, t = self.status(stream)
        if p:
            raise MergePoisoned("IpcMerge rank %d: merge poisoned (%d phase waits timed out here; a peer died, "
                                "stalled past %d ms or was poisoned itself); the merged ranges are all-ones"
                                % (self.rank, t, self.timeout_ms))

    def close(self, check=True):
        """Unmaps the peers (after a barrier: no peer reads my words any more);
        raises MergePoisoned if the merge was poisoned, unless check=False."""
        torch.cuda.synchronize(self.words.device)
        dist.barrier(group=self.group)
        poisoned, n = self.status()
        for b in self.bases:
            self.ctx.ipc_close(b)
        self.bases, self.ptrs, self.fptrs = [], [], []
        if poisoned and check:
            raise MergePoisoned("IpcMerge: merge poisoned, %d phase waits timed out on this rank" % n)

    def _phase_done(self, stream):
        stream.synchronize()
        dist.barrier(group=self.group)

    def _check_range(self, lo, hi):
        """The peer loads use raw pointers into the other ranks' words: every
        rank must merge the same range.  Checked once per distinct range (the
        ranks see the same sequence of ranges, so they agree on which are new)."""
        if (lo, hi) in self._checked:
            return
        rng = torch.tensor([lo, hi, -lo, -hi], dtype=torch.int64)
        dist.all_reduce(rng, op=dist.ReduceOp.MAX, group=self.group)
        if rng.tolist() != [lo, hi, -lo, -hi]:
            raise ValueError("ranks disagree on the word range: this rank [%d, %d)" % (lo, hi))
        self._checked.add((lo, hi))

    def allreduce(self, lo=0, hi=None, stream=None, check=False):
        """In-place OR-allreduce of words[lo:hi] (word indices) over the group,
        after the caller's pending work on `stream` (default: current).
        ordered="device": enqueued only (returns at once); the stream's later
        work sees the merged range.  ordered="host": returns when every rank's
        range is merged.  check=True: also waits for the stream and raises
        MergePoisoned if the merge (or an earlier one) was poisoned."""
        hi = self.words.numel() if hi is None else hi
        if not 0 <= lo <= hi <= self.words.numel():
            raise ValueError("word range [%d, %d) outside this rank's %d words" % (lo, hi, self.words.numel()))
        self._check_range(lo, hi)
        stream = stream or torch.cuda.current_stream(self.words.device)
        if self.ordered == "host":
            self._phase_done(stream)  # every partial of the range is final
            for op in merge_schedule(self.rank, self.world, lo, hi, 0):
                if op[0] in ("gather", "copy"):
                    self._gather(op, stream)
                elif op[0] == "wait" and op[1] in (1, 2):
                    self._phase_done(stream)
        else:
            self.epoch += 1
            poison = [p + 4 * _POISON for p in self.fptrs]
            for op in merge_schedule(self.rank, self.world, lo, hi, self.epoch):
                if op[0] == "signal":
                    _, ph, e = op
                    self.ctx.flag_signal_dev(self.fptrs[self.rank] + 4 * ph, e, stream=stream.cuda_stream)
                elif op[0] == "wait":
                    _, ph, e = op
                    self.ctx.flag_wait_dev([p + 4 * ph for p in self.fptrs], e, self.status_ptr, self.timeout_ms,
                                           poison_ptrs=poison, stream=stream.cuda_stream)
                elif op[0] == "fill":
                    _, a, b = op
                    self.ctx.poison_fill_dev(self.ptrs[self.rank] + 8 * a, b - a, self.status_ptr,
                                             stream=stream.cuda_stream)
                else:
                    self._gather(op, stream)
        if check:
            self.check(stream)
        return self.words

    def _gather(self, op, stream):
        if op[0] == "gather":
            _, a, b, srcs = op
            self.ctx.or_gather_dev(self.ptrs[self.rank] + 8 * a, [self.ptrs[r] + 8 * a for r in srcs], b - a,
                                   stream=stream.cuda_stream, status_ptr=self.status_ptr)
        else:  # "copy": every other rank's merged slice in one kernel
            _, lo, hi, per, srcs = op
            ptrs = [self.ptrs[r] + 8 * lo if r in srcs else 0 for r in range(self.world)]
            self.ctx.copy_slices_dev(self.ptrs[self.rank] + 8 * lo, ptrs, per, hi - lo, stream=stream.cuda_stream,
                                     status_ptr=self.status_ptr)


def merge_schedule(rank, world, lo, hi, epoch):
    """The device-ordered merge of words[lo:hi] as this rank's stream sees it,
    in order: ("signal", phase, epoch) — set my flag[phase] = epoch;
    ("wait", phase, epoch) — until every rank's flag[phase] >= epoch (a
    timeout, or any rank's poison word set, poisons this merge instead);
    ("gather", a, b, ranks) — my words[a:b] = OR of those ranks' words[a:b]
    (my own index among them: in place); ("copy", lo, hi, per, ranks) — for
    each listed rank r, my words of slice r (words [lo + r per, lo + (r+1) per)
    within [lo, hi)) = rank r's (lsmb_copy_slices_dev: one kernel, every peer
    link at once); ("fill", lo, hi) — my words[lo:hi] = all-ones if this merge
    is poisoned.  A poisoned gather / copy writes all-ones and reads no peer.
    Phase 0: every partial of the range is final; 1: every slice merged; 2:
    every rank holds the merged range."""
    per = _slices(hi - lo, world)
    sl = [(min(hi, lo + r * per), min(hi, lo + (r + 1) * per)) for r in range(world)]
    ops = [("signal", 0, epoch), ("wait", 0, epoch)]
    a, b = sl[rank]
    if b > a:
        ops.append(("gather", a, b, list(range(world))))
    ops += [("signal", 1, epoch), ("wait", 1, epoch)]
    peers = [r for r, (a, b) in enumerate(sl) if r != rank and b > a]
    if peers:
        ops.append(("copy", lo, hi, per, peers))
    ops += [("signal", 2, epoch), ("wait", 2, epoch)]
    if hi > lo:
        ops.append(("fill", lo, hi))
    return ops
