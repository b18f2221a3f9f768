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
    `group` (gloo) only orders the phases: a host barrier after each rank's
    stream finished the previous phase, and one at the end so that no rank
    rewrites its words while a peer may still read them.  Per GPU it reads
    (G-1)/G of the range twice over the peer links, the RCCL path's bytes."""

    def __init__(self, words, ctx, group=None):
        import lsmbloom
        self.words, self.ctx, self.group = words, ctx, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        h, off = lsmbloom.ipc_export(words)
        allh = [None] * self.world
        dist.all_gather_object(allh, (h, off, words.numel(), words.device.index), group=group)
        self.bases, self.ptrs = [], []
        for r, (hh, oo, n, _) in enumerate(allh):
            if n != words.numel():
                raise ValueError("rank %d's words hold %d words, mine %d" % (r, n, words.numel()))
            if r == self.rank:
                self.ptrs.append(words.data_ptr())
            else:
                base = ctx.ipc_import(hh)
                self.bases.append(base)
                self.ptrs.append(base + oo)

    def close(self):
        dist.barrier(group=self.group)  # no peer reads my words any more
        for b in self.bases:
            self.ctx.ipc_close(b)
        self.bases, self.ptrs = [], []

    def _phase_done(self, stream):
        stream.synchronize()
        dist.barrier(group=self.group)

    def allreduce(self, lo=0, hi=None, stream=None):
        """In-place OR-allreduce of words[lo:hi] (word indices) over the group.
        The caller's pending work on `stream` (default: current) that writes
        words[lo:hi] is waited for first; returns when every rank's range is
        merged (host-synchronous)."""
        hi = self.words.numel() if hi is None else hi
        if not 0 <= lo <= hi <= self.words.numel():
            raise ValueError("word range [%d, %d) outside this rank's %d words" % (lo, hi, self.words.numel()))
        stream = stream or torch.cuda.current_stream(self.words.device)
        stream.synchronize()
        # every partial of the range is final; the exchange that orders this
        # phase also checks that every rank merges the same range (the peer
        # loads use raw pointers into the other ranks' words)
        rng = torch.tensor([lo, hi, -lo, -hi], dtype=torch.int64)
        dist.all_reduce(rng, op=dist.ReduceOp.MAX, group=self.group)
        if rng.tolist() != [lo, hi, -lo, -hi]:
            raise ValueError("ranks disagree on the word range: this rank [%d, %d)" % (lo, hi))
        per = _slices(hi - lo, self.world)
        sl = [(min(hi, lo + r * per), min(hi, lo + (r + 1) * per)) for r in range(self.world)]
        a, b = sl[self.rank]
        if b > a:
            self.ctx.or_gather_dev(self.ptrs[self.rank] + 8 * a, [p + 8 * a for p in self.ptrs], b - a,
                                   stream=stream.cuda_stream)
        self._phase_done(stream)  # every slice merged
        for r, (a, b) in enumerate(sl):
            if r != self.rank and b > a:
                self.ctx.or_gather_dev(self.ptrs[self.rank] + 8 * a, [self.ptrs[r] + 8 * a], b - a,
                                       stream=stream.cuda_stream)
        self._phase_done(stream)  # every rank holds the merged range; words may be rewritten
        return self.words
