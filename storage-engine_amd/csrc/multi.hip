// multi.hip — one process, several GPUs: a sharded build merged over xGMI.
//
// The store flushes and compacts from one process (src/db/mod.rs:377-383,
// src/compaction/scheduler.rs:150-158, both through SSTableBuilder::add,
// src/sstable/builder.rs:93).  When one run's key set is large, lsmb_multi
// splits it into G contiguous shards, builds a full-size partial filter per
// shard on its own GPU, and merges the partials with a bitwise-OR
// reduce-scatter done by peer loads: shard g's GPU reads word-slice g of every
// partial straight out of the other GPUs' HBM over xGMI and ORs it (no staging
// copy, every peer link busy at once).  OR is associative, commutative and
// idempotent, so the merged filter is bit-identical to a single-GPU build of
// the whole run.  RCCL has no bitwise-OR reduction (rccl.h ncclRedOp_t), and
// inside one process peer loads need no communicator at all.
//
//   device-resident (lsmb_multi_build_fixed_dev): + all-gather of the merged
//     slices, so every GPU ends up holding the whole filter;
//   host keys -> serialized block (lsmb_multi_build_block): each GPU uploads
//     its own shard (G PCIe links in parallel) and copies only its merged
//     slice into the block (again G links in parallel); no all-gather.
//
// Shards may name the same device more than once (tests on a one-GPU box run
// G = 2..4 shards on device 0: the same kernels and the same merge, with the
// "peer" reads served locally).
#include <stdarg.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "ctx.hpp"

using namespace lsmb;

namespace {

constexpr int kMaxShards = 16;

struct OrSources {
    const void* p[kMaxShards];
    uint32_t n;
};

// The merge's fail-safe (round 6).  `status` (may be null) is the merge's
// status words: status[0] != 0 = poisoned (a phase wait timed out or saw a
// peer's poison; k_flag_wait).  A poisoned merge must not read its peers'
// words (they may be mid-rewrite) and must never leave a bit unset that the
// true merge would set: it writes all-ones instead, the one value that is a
// superset of every partial, so the filter then answers "maybe" for every key
// (false positives only, never a false negative: src/sstable/reader.rs:196-199).
__device__ __forceinline__ bool poisoned(const uint32_t* status) {
    return status && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

template <class V>
__device__ __forceinline__ V all_ones() {
    if constexpr (sizeof(V) == 16) {
        return V{~0u, ~0u, ~0u, ~0u};
    } else {
        return ~V(0);
    }
}

// dst[i] = OR over j of src_j[i], i < count (elements of V).  dst may be one
// of the sources (the owner's own partial): each element is read by every
// source load before its one store, by the same thread.  So dst is not
// __restrict__ (it aliases a source).  N > 0: N sources known at compile
// time, so a thread's N loads (over N peer links) are all in flight before
// the first OR; N = 0: a runtime count (9..16 sources).  Poisoned: all-ones.
template <class V, int N>
__global__ __launch_bounds__(256) void k_or_gather(V* dst, OrSources src, uint64_t count, const uint32_t* status) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (poisoned(status)) {
        for (; i < count; i += stride) dst[i] = all_ones<V>();
        return;
    }
    auto orv = [](V& v, const V& x) {
        if constexpr (sizeof(V) == 16) {
            v.x |= x.x, v.y |= x.y, v.z |= x.z, v.w |= x.w;
        } else {
            v |= x;
        }
    };
    for (; i < count; i += stride) {
        V v = static_cast<const V*>(src.p[0])[i];
        if constexpr (N > 0) {
            V w[N];
#pragma unroll
            for (int j = 1; j < N; j++) w[j] = static_cast<const V*>(src.p[j])[i];
#pragma unroll
            for (int j = 1; j < N; j++) orv(v, w[j]);
        } else {
            for (uint32_t j = 1; j < src.n; j++) orv(v, static_cast<const V*>(src.p[j])[i]);
        }
        dst[i] = v;
    }
}

// The all-gather of a merge in one kernel: dst[i] = src_r[i] for every
// element of slice r = [r per, min((r+1) per, count)) whose source is set
// (src.p[r] == nullptr: the caller's own slice, left alone).  blockIdx.y is
// the slice, so every peer link streams at once (one copy per peer, one
// after another on a stream, would use one link at a time).  Four elements
// in flight per thread.  Poisoned: the slices are written all-ones.
template <class V>
__global__ __launch_bounds__(256) void k_copy_slices(V* __restrict__ dst, OrSources src, uint64_t per, uint64_t count,
                                                     const uint32_t* status) {
    const V* __restrict__ s = static_cast<const V*>(src.p[blockIdx.y]);
    if (!s) return;  // (block-uniform)
    const uint64_t a = (uint64_t)blockIdx.y * per, b = min(count, a + per);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = a + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (poisoned(status)) {
        for (; i < b; i += stride) dst[i] = all_ones<V>();
        return;
    }
    for (; i + 3 * stride < b; i += 4 * stride) {
        V x[4];
#pragma unroll
        for (int u = 0; u < 4; u++) x[u] = s[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; u++) dst[i + u * stride] = x[u];
    }
    for (; i < b; i += stride) dst[i] = s[i];
}

// The merge's last step: a merge that ended poisoned (at any of its waits,
// the last included) leaves its whole range all-ones.  Not poisoned: every
// block reads the status word and ends.
__global__ __launch_bounds__(256) void k_poison_fill(uint64_t* words, uint64_t count, const uint32_t* status) {
    if (!poisoned(status)) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) words[i] = ~0ull;
}

// ---- device-ordered phase flags (cross-process merge, lsmb_flag_*) --------
// A flag is a u32 epoch counter in device memory (this process's, or a peer's
// mapped over IPC).  signal: one system-scope release store of the epoch after
// everything before it on the stream (kernel boundaries already release each
// kernel's stores at agent scope, i.e. L2 written back across the XCDs).
// wait: one wave, lane j polls flag j with system-scope loads (no stale L2
// copy) until every flag reaches the epoch (wrap-safe compare), backing off
// with s_sleep.  The wait is the merge's fail-safe (round 6):
//   * it gives up after `ticks` of the constant-rate wall clock (a peer that
//     died cannot hang the queue), counts the timeout in status[1] and
//     poisons the merge (status[0] = 1, a system-scope store: the status
//     words sit in the flag array the peers map, so they see it);
//   * it also ends as soon as any rank's poison word (poison[j], this rank's
//     own among them) is set, and reads every poison word once more after the
//     flags were met: a peer that gave up on us may already be rewriting the
//     words we read, and its poison is published before that rewrite, so the
//     next wait after such a read sees it and poisons this merge too.
// A poisoned merge writes all-ones instead of reading peers (k_or_gather,
// k_copy_slices) and ends with its range all-ones (k_poison_fill).
constexpr uint32_t kMaxFlags = 64;
struct FlagSet {
    const uint32_t* p[kMaxFlags];
    uint32_t n;
};

__global__ __launch_bounds__(64) void k_flag_signal(uint32_t* flag, uint32_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t load_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_flag_wait(FlagSet fs, FlagSet ps, uint32_t value, uint64_t ticks,
                                                  uint32_t* status) {
    const uint32_t j = threadIdx.x;
    // the loop is wave-uniform: its exits are ballots and the scalar wall clock
    bool met = j >= fs.n;
    bool timed_out = false, poison = false;
    const uint64_t t0 = (uint64_t)wall_clock64();
    for (;;) {
        if (!met) met = (int32_t)(load_sys(fs.p[j]) - value) >= 0;
        const bool pz = j < ps.n && load_sys(ps.p[j]) != 0;
        if (__ballot(pz)) {
            poison = true;
            break;
        }
        if (__ballot(!met) == 0) break;
        if ((uint64_t)wall_clock64() - t0 > ticks) {
            timed_out = true;
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
    if (!poison && __ballot(j < ps.n && load_sys(ps.p[j]) != 0)) poison = true;
    if (j == 0 && (timed_out || poison)) {
        if (timed_out) atomicAdd(&status[1], 1u);
        __hip_atomic_store(&status[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: later reads see the peers' data
}

template <class V>
hipError_t or_gather_n(V* dst, const OrSources& s, uint64_t count, uint32_t g, const uint32_t* status, hipStream_t st) {
    const dim3 grid(g), block(256);
    switch (s.n) {
        case 1: k_or_gather<V, 1><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 2: k_or_gather<V, 2><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 3: k_or_gather<V, 3><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 4: k_or_gather<V, 4><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 5: k_or_gather<V, 5><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 6: k_or_gather<V, 6><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 7: k_or_gather<V, 7><<<grid, block, 0, st>>>(dst, s, count, status); break;
        case 8: k_or_gather<V, 8><<<grid, block, 0, st>>>(dst, s, count, status); break;
        default: k_or_gather<V, 0><<<grid, block, 0, st>>>(dst, s, count, status); break;
    }
    return hipGetLastError();
}

hipError_t launch_or_gather(uint64_t* dst, const OrSources& s, uint64_t nwords, int num_cus, hipStream_t st,
                            const uint32_t* status = nullptr) {
    if (nwords == 0) return hipSuccess;
    bool a16 = ((uintptr_t)dst & 15) == 0 && (nwords & 1) == 0;
    for (uint32_t j = 0; j < s.n; j++) a16 = a16 && ((uintptr_t)s.p[j] & 15) == 0;
    const uint64_t count = a16 ? nwords / 2 : nwords;
    uint64_t g = (count + 255) / 256;
    g = std::min<uint64_t>(g, (uint64_t)num_cus * 8);
    if (g < 1) g = 1;
    if (a16) return or_gather_n((uint4*)dst, s, count, (uint32_t)g, status, st);
    return or_gather_n(dst, s, count, (uint32_t)g, status, st);
}

// dst words of slice r (slice_words each, nwords in all) from s.p[r] where set.
hipError_t launch_copy_slices(uint64_t* dst, const OrSources& s, uint64_t slice_words, uint64_t nwords, int num_cus,
                              hipStream_t st, const uint32_t* status = nullptr) {
    if (nwords == 0 || s.n == 0) return hipSuccess;
    bool a16 = ((uintptr_t)dst & 15) == 0 && (nwords & 1) == 0 && (slice_words & 1) == 0;
    for (uint32_t j = 0; j < s.n; j++) a16 = a16 && ((uintptr_t)s.p[j] & 15) == 0;
    const uint64_t per = a16 ? slice_words / 2 : slice_words, count = a16 ? nwords / 2 : nwords;
    uint64_t gx = (per + 1023) / 1024;  // 256 threads x 4 elements per block
    gx = std::min<uint64_t>(gx, std::max<uint64_t>(1, (uint64_t)num_cus * 8 / s.n));
    if (gx < 1) gx = 1;
    const dim3 grid((uint32_t)gx, s.n);
    if (a16)
        k_copy_slices<uint4><<<grid, dim3(256), 0, st>>>((uint4*)dst, s, per, count, status);
    else
        k_copy_slices<uint64_t><<<grid, dim3(256), 0, st>>>(dst, s, per, count, status);
    return hipGetLastError();
}

}  // namespace

struct lsmb_multi {
    std::vector<lsmb_ctx*> ctx;  // one per shard
    std::vector<hipStream_t> mst;                 // per shard: merge stream (device builds overlap it)
    std::vector<hipEvent_t> ev_built, ev_merged;  // per shard, recorded on the shard's stream
    std::vector<hipEvent_t> t0, t1, t2;           // timing per shard: start, built, merged
    std::vector<DevBuf> words;                    // per-shard device words (host-key builds)
    bool timed = false;
};

namespace {

int shards(const lsmb_multi* m) { return (int)m->ctx.size(); }

// Word-slice g of an nw-word filter: [g*per, min((g+1)*per, nw)), per even so
// every slice starts 16-B aligned.
uint64_t slice_words(uint64_t nw, int G) {
    uint64_t per = (nw + G - 1) / G;
    return (per + 1) & ~1ull;
}

void slice_of(uint64_t nw, int G, int g, uint64_t* lo, uint64_t* hi) {
    const uint64_t per = slice_words(nw, G);
    *lo = std::min<uint64_t>(nw, (uint64_t)g * per);
    *hi = std::min<uint64_t>(nw, (uint64_t)(g + 1) * per);
}

// Runs f(g) for every shard on its own host thread (each sets its device);
// returns the first failure with its message.
template <class F>
int for_shards(lsmb_multi* m, F&& f) {
    const int G = shards(m);
    std::vector<int> rc(G, LSMB_OK);
    std::vector<std::string> msg(G);
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++)
        th.emplace_back([&, g]() {
            DevGuard dg(m->ctx[g]->dev);
            rc[g] = f(g);
            if (rc[g]) msg[g] = last_error();
        });
    for (auto& t : th) t.join();
    for (int g = 0; g < G; g++)
        if (rc[g]) {
            set_last_error("shard " + std::to_string(g) + ": " + msg[g]);
            return rc[g];
        }
    return LSMB_OK;
}

// The stream shard g merges on: its build stream, or (overlapped device
// builds) its merge stream.
hipStream_t merge_stream(lsmb_multi* m, int g, bool side) { return side ? m->mst[g] : m->ctx[g]->st; }

// Reduce-scatter of words [base, base + nw): after every shard's build
// (ev_built), shard g ORs sub-slice g of all partials into its own partial.
// `part[j]` = shard j's words (device of j).
int merge_reduce_scatter(lsmb_multi* m, uint64_t* const* part, uint64_t nw, uint64_t base = 0, bool side = false) {
    const int G = shards(m);
    for (int g = 0; g < G; g++) {
        lsmb_ctx* c = m->ctx[g];
        DevGuard dg(c->dev);
        const hipStream_t st = merge_stream(m, g, side);
        for (int j = 0; j < G; j++)
            if (j != g || side) HIP_TRY(hipStreamWaitEvent(st, m->ev_built[j], 0));
        uint64_t lo, hi;
        slice_of(nw, G, g, &lo, &hi);
        lo += base, hi += base;
        OrSources s;
        s.n = (uint32_t)G;
        for (int j = 0; j < G; j++) s.p[j] = part[j] + lo;
        HIP_TRY(launch_or_gather(part[g] + lo, s, hi - lo, c->num_cus, st));
        HIP_TRY(hipEventRecord(m->ev_merged[g], st));
    }
    return LSMB_OK;
}

// All-gather of words [base, base + nw): shard g copies every other shard's
// merged sub-slice into its words, all of them in one kernel of peer loads
// (every peer link at once).
int merge_all_gather(lsmb_multi* m, uint64_t* const* part, uint64_t nw, uint64_t base = 0, bool side = false) {
    const int G = shards(m);
    const uint64_t per = slice_words(nw, G);
    for (int g = 0; g < G; g++) {
        lsmb_ctx* c = m->ctx[g];
        DevGuard dg(c->dev);
        const hipStream_t st = merge_stream(m, g, side);
        OrSources s;
        s.n = (uint32_t)G;
        for (int j = 0; j < G; j++) {
            s.p[j] = j == g ? nullptr : part[j] + base;
            if (j != g) HIP_TRY(hipStreamWaitEvent(st, m->ev_merged[j], 0));
        }
        HIP_TRY(launch_copy_slices(part[g] + base, s, per, nw, c->num_cus, st));
    }
    return LSMB_OK;
}

int sync_all(lsmb_multi* m) {
    for (lsmb_ctx* c : m->ctx) {
        DevGuard dg(c->dev);
        HIP_TRY(hipStreamSynchronize(c->st));
    }
    return LSMB_OK;
}

}  // namespace

extern "C" {

int lsmb_multi_open(lsmb_multi** out, const int* devices, int ndev) {
    if (!out) return fail(LSMB_EINVAL, "null lsmb_multi pointer");
    *out = nullptr;
    if (ndev < 1 || ndev > kMaxShards) return fail(LSMB_EINVAL, "ndev must be in [1, %d]", kMaxShards);
    lsmb_multi* m = new lsmb_multi;
    for (int g = 0; g < ndev; g++) {
        lsmb_ctx* c = nullptr;
        const int d = devices ? devices[g] : g;
        if (int rc = lsmb_open(&c, d)) {
            lsmb_multi_close(m);
            return rc;
        }
        m->ctx.push_back(c);
    }
    // Peer access between every pair of distinct devices: the merge kernel
    // reads the other GPUs' partials in place.
    for (int g = 0; g < ndev; g++) {
        DevGuard dg(m->ctx[g]->dev);
        for (int j = 0; j < ndev; j++) {
            const int a = m->ctx[g]->dev, b = m->ctx[j]->dev;
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
                lsmb_multi_close(m);
                return fail(LSMB_ENODEV, "device %d cannot access device %d's memory (no xGMI peer path)", a, b);
            }
            hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e == hipErrorPeerAccessAlreadyEnabled) {
                (void)hipGetLastError();
            } else if (e != hipSuccess) {
                lsmb_multi_close(m);
                return hip_fail(e, "hipDeviceEnablePeerAccess");
            }
        }
        m->mst.push_back(nullptr);
        if (hipStreamCreateWithFlags(&m->mst[g], hipStreamNonBlocking) != hipSuccess) {
            lsmb_multi_close(m);
            return fail(LSMB_EHIP, "merge stream creation failed on device %d", m->ctx[g]->dev);
        }
        m->ev_built.push_back(nullptr);
        m->ev_merged.push_back(nullptr);
        m->t0.push_back(nullptr);
        m->t1.push_back(nullptr);
        m->t2.push_back(nullptr);
        if (hipEventCreateWithFlags(&m->ev_built[g], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&m->ev_merged[g], hipEventDisableTiming) != hipSuccess ||
            hipEventCreate(&m->t0[g]) != hipSuccess || hipEventCreate(&m->t1[g]) != hipSuccess ||
            hipEventCreate(&m->t2[g]) != hipSuccess) {
            lsmb_multi_close(m);
            return fail(LSMB_EHIP, "event creation failed on device %d", m->ctx[g]->dev);
        }
    }
    m->words.resize(ndev);
    *out = m;
    return LSMB_OK;
}

void lsmb_multi_close(lsmb_multi* m) {
    if (!m) return;
    for (size_t g = 0; g < m->ctx.size(); g++) {
        DevGuard dg(m->ctx[g]->dev);
        hipStreamSynchronize(m->ctx[g]->st);
        if (g < m->mst.size() && m->mst[g]) hipStreamSynchronize(m->mst[g]), hipStreamDestroy(m->mst[g]);
        for (auto* v : {&m->ev_built, &m->ev_merged, &m->t0, &m->t1, &m->t2})
            if (g < v->size() && (*v)[g]) hipEventDestroy((*v)[g]);
        if (g < m->words.size()) m->words[g].release();
    }
    for (lsmb_ctx* c : m->ctx) lsmb_close(c);
    delete m;
}

int lsmb_multi_size(const lsmb_multi* m) { return m ? shards(m) : 0; }

lsmb_ctx* lsmb_multi_ctx(lsmb_multi* m, int shard) {
    if (!m || shard < 0 || shard >= shards(m)) return nullptr;
    return m->ctx[shard];
}

int lsmb_multi_build_fixed_dev(lsmb_multi* m, const void* const* d_keys, const uint64_t* n, uint32_t key_len,
                               uint32_t num_bits, uint32_t k, void* const* d_words) {
    if (!m || !d_keys || !n || !d_words) return fail(LSMB_EINVAL, "null argument");
    if (int rc = check_filter(num_bits, k)) return rc;
    const int G = shards(m);
    const uint64_t nw = nwords64(num_bits);
    for (int g = 0; g < G; g++)
        if (!d_words[g] || (n[g] && !d_keys[g])) return fail(LSMB_EINVAL, "null device pointer (shard %d)", g);
    // Partitioned builds of big filters run in sweeps (lsmb_build_sweeps); sweep
    // s completes one word range.  Per sweep: every shard builds it on its
    // build stream (asynchronous), then the range is reduce-scattered and
    // all-gathered on the shards' merge streams while sweep s + 1 builds.
    uint64_t nmax = 0;
    for (int g = 0; g < G; g++) nmax = std::max(nmax, n[g]);
    const int nsw = (G > 1 && k) ? lsmb_build_sweeps(num_bits, k, nmax) : 1;
    std::vector<uint64_t*> part(G);
    for (int g = 0; g < G; g++) part[g] = (uint64_t*)d_words[g];
    for (int g = 0; g < G; g++) {
        DevGuard dg(m->ctx[g]->dev);
        HIP_TRY(hipEventRecord(m->t0[g], m->ctx[g]->st));
    }
    for (int sw = 0; sw < nsw; sw++) {
        for (int g = 0; g < G; g++) {
            lsmb_ctx* c = m->ctx[g];
            DevGuard dg(c->dev);
            if (n[g] && k) {
                KeyBatch kb{(const uint8_t*)d_keys[g], nullptr, key_len, key_len ? n[g] : 1};
                if (int rc = build_dev(c, kb, num_bits, k, (uint32_t*)d_words[g], c->st, nsw > 1 ? sw : -1)) return rc;
            }
            if (sw + 1 == nsw) HIP_TRY(hipEventRecord(m->t1[g], c->st));
            HIP_TRY(hipEventRecord(m->ev_built[g], c->st));
        }
        if (G > 1) {
            uint64_t lo = 0, hi = nw;
            if (nsw > 1 && lsmb_sweep_words(num_bits, k, nmax, sw, &lo, &hi)) return LSMB_EINVAL;
            const bool side = nsw > 1;
            if (int rc = merge_reduce_scatter(m, part.data(), hi - lo, lo, side)) return rc;
            if (int rc = merge_all_gather(m, part.data(), hi - lo, lo, side)) return rc;
        }
    }
    for (int g = 0; g < G; g++) {
        lsmb_ctx* c = m->ctx[g];
        DevGuard dg(c->dev);
        if (nsw > 1 && G > 1) {  // the build stream takes the merges back: callers sync on it
            HIP_TRY(hipEventRecord(m->ev_merged[g], m->mst[g]));
            HIP_TRY(hipStreamWaitEvent(c->st, m->ev_merged[g], 0));
        }
        HIP_TRY(hipEventRecord(m->t2[g], c->st));
    }
    m->timed = true;
    return sync_all(m);
}

int lsmb_multi_build_block(lsmb_multi* m, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                           uint32_t num_bits, uint32_t k, uint8_t* block, uint64_t block_len) {
    if (!m || !block) return fail(LSMB_EINVAL, "null argument");
    if (int rc = check_filter(num_bits, k)) return rc;
    const uint64_t nw = nwords64(num_bits);
    if (block_len < 12 + 8 * nw) return fail(LSMB_EINVAL, "block buffer too small");
    if (n && !offsets && !data && key_len) return fail(LSMB_EINVAL, "null keys");
    if (n && offsets)
        for (uint64_t i = 0; i < n; i++)
            if (offsets[i + 1] < offsets[i]) return fail(LSMB_EINVAL, "offsets not non-decreasing at %llu", (unsigned long long)i);
    // header of BloomFilter::serialize (src/bloom/mod.rs:102-115)
    const uint32_t hdr[3] = {k, num_bits, (uint32_t)nw};
    for (int i = 0; i < 3; i++)
        for (int b = 0; b < 4; b++) block[4 * i + b] = (uint8_t)(hdr[i] >> (8 * b));
    if (n == 0 || k == 0) {
        memset(block + 12, 0, nw * 8);
        return LSMB_OK;
    }
    const int G = shards(m);
    std::vector<uint64_t*> part(G);
    // 1. per shard (own thread: the H2D loops run in parallel over G PCIe links):
    //    zeroed words, chunked H2D of the shard's keys overlapped with its build
    if (!offsets && key_len == 0) n = 1;  // every key is the empty key: one insert
    int rc = for_shards(m, [&](int g) -> int {
        lsmb_ctx* c = m->ctx[g];
        HIP_TRY(m->words[g].ensure(std::max<uint64_t>(nw, 2) * 8));
        part[g] = (uint64_t*)m->words[g].p;
        HIP_TRY(hipEventRecord(m->t0[g], c->st));
        HIP_TRY(hipMemsetAsync(part[g], 0, nw * 8, c->st));
        const uint64_t lo = n * g / G, hi = n * (g + 1) / G;
        if (hi > lo) {
            if (offsets) {
                if (int r = host_build_dev(c, data, offsets + lo, 0, hi - lo, num_bits, k, (uint32_t*)part[g])) return r;
            } else {
                if (int r = host_build_dev(c, data + lo * key_len, nullptr, key_len, hi - lo, num_bits, k,
                                           (uint32_t*)part[g]))
                    return r;
            }
        }
        HIP_TRY(hipEventRecord(m->t1[g], c->st));
        HIP_TRY(hipEventRecord(m->ev_built[g], c->st));
        return LSMB_OK;
    });
    if (rc) return rc;
    // 2. OR reduce-scatter (peer loads); 3. each shard copies its merged slice
    //    into the block body (no all-gather: the host only needs each slice once)
    if (G > 1)
        if (int r = merge_reduce_scatter(m, part.data(), nw)) return r;
    rc = for_shards(m, [&](int g) -> int {
        lsmb_ctx* c = m->ctx[g];
        uint64_t lo, hi;
        slice_of(nw, G, g, &lo, &hi);
        if (hi > lo)
            HIP_TRY(hipMemcpyAsync(block + 12 + lo * 8, part[g] + lo, (hi - lo) * 8, hipMemcpyDeviceToHost, c->st));
        HIP_TRY(hipEventRecord(m->t2[g], c->st));
        HIP_TRY(hipStreamSynchronize(c->st));
        return LSMB_OK;
    });
    m->timed = rc == LSMB_OK;
    return rc;
}

// ---- one process per GPU: IPC mappings + the peer-load OR gather
int lsmb_ipc_export(const void* d_ptr, uint8_t* handle, uint64_t* offset) {
    if (!d_ptr || !handle || !offset) return fail(LSMB_EINVAL, "null argument");
    static_assert(sizeof(hipIpcMemHandle_t) == LSMB_IPC_HANDLE_BYTES, "IPC handle size");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    HIP_TRY(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_ptr));
    hipIpcMemHandle_t h;
    HIP_TRY(hipIpcGetMemHandle(&h, (void*)base));
    memcpy(handle, &h, sizeof h);
    *offset = (uint64_t)((const char*)d_ptr - (const char*)base);
    return LSMB_OK;
}

int lsmb_ipc_import(lsmb_ctx* c, const uint8_t* handle, void** d_base) {
    if (!c || !handle || !d_base) return fail(LSMB_EINVAL, "null argument");
    *d_base = nullptr;
    DevGuard g(c->dev);
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof h);
    const hipError_t e = hipIpcOpenMemHandle(d_base, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *d_base = nullptr;
        return fail(e == hipErrorInvalidContext || e == hipErrorInvalidValue ? LSMB_EINVAL : LSMB_EHIP,
                    "hipIpcOpenMemHandle: %s (a handle of this same process cannot be opened)", hipGetErrorString(e));
    }
    return LSMB_OK;
}

int lsmb_ipc_close(lsmb_ctx* c, void* d_base) {
    if (!c || !d_base) return fail(LSMB_EINVAL, "null argument");
    DevGuard g(c->dev);
    HIP_TRY(hipIpcCloseMemHandle(d_base));  // teardown of a mapping, no device memory freed
    return LSMB_OK;
}

int lsmb_or_gather_dev(lsmb_ctx* c, void* d_dst, const void* const* d_srcs, uint32_t nsrc, uint64_t nwords,
                       const uint32_t* d_status, void* stream) {
    if (!c || !d_srcs) return fail(LSMB_EINVAL, "null argument");
    if (nsrc < 1 || nsrc > (uint32_t)kMaxShards) return fail(LSMB_EINVAL, "nsrc must be in [1, %d]", kMaxShards);
    if (nwords == 0) return LSMB_OK;
    if (!d_dst) return fail(LSMB_EINVAL, "null device pointer");
    OrSources s;
    s.n = nsrc;
    for (uint32_t j = 0; j < nsrc; j++) {
        if (!d_srcs[j]) return fail(LSMB_EINVAL, "null source %u", j);
        if (((uintptr_t)d_srcs[j] & 7) != 0) return fail(LSMB_EINVAL, "source %u is not 8-byte aligned", j);
        s.p[j] = d_srcs[j];
    }
    if (((uintptr_t)d_dst & 7) != 0) return fail(LSMB_EINVAL, "d_dst is not 8-byte aligned");
    if (((uintptr_t)d_status & 3) != 0) return fail(LSMB_EINVAL, "d_status is not 4-byte aligned");
    DevGuard g(c->dev);
    HIP_TRY(launch_or_gather((uint64_t*)d_dst, s, nwords, c->num_cus, pick_stream(c, stream), d_status));
    return LSMB_OK;
}

int lsmb_copy_slices_dev(lsmb_ctx* c, void* d_dst, const void* const* d_srcs, uint32_t nsrc, uint64_t slice_words,
                         uint64_t nwords, const uint32_t* d_status, void* stream) {
    if (!c || !d_srcs) return fail(LSMB_EINVAL, "null argument");
    if (nsrc < 1 || nsrc > (uint32_t)kMaxShards) return fail(LSMB_EINVAL, "nsrc must be in [1, %d]", kMaxShards);
    if (nwords == 0) return LSMB_OK;
    if (!d_dst) return fail(LSMB_EINVAL, "null device pointer");
    if (slice_words == 0 || (slice_words * nsrc < nwords)) return fail(LSMB_EINVAL, "nsrc slices of slice_words must cover nwords");
    OrSources s;
    s.n = nsrc;
    for (uint32_t j = 0; j < nsrc; j++) {
        if (d_srcs[j] && ((uintptr_t)d_srcs[j] & 7) != 0) return fail(LSMB_EINVAL, "source %u is not 8-byte aligned", j);
        s.p[j] = d_srcs[j];
    }
    if (((uintptr_t)d_dst & 7) != 0) return fail(LSMB_EINVAL, "d_dst is not 8-byte aligned");
    if (((uintptr_t)d_status & 3) != 0) return fail(LSMB_EINVAL, "d_status is not 4-byte aligned");
    DevGuard g(c->dev);
    HIP_TRY(launch_copy_slices((uint64_t*)d_dst, s, slice_words, nwords, c->num_cus, pick_stream(c, stream), d_status));
    return LSMB_OK;
}

int lsmb_poison_fill_dev(lsmb_ctx* c, void* d_words, uint64_t nwords, const uint32_t* d_status, void* stream) {
    if (!c || !d_status) return fail(LSMB_EINVAL, "null argument");
    if (nwords == 0) return LSMB_OK;
    if (!d_words || ((uintptr_t)d_words & 7) != 0) return fail(LSMB_EINVAL, "d_words: null or not 8-byte aligned");
    if (((uintptr_t)d_status & 3) != 0) return fail(LSMB_EINVAL, "d_status is not 4-byte aligned");
    DevGuard g(c->dev);
    // a small grid: when the merge is healthy every block only reads the status
    const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((nwords + 255) / 256, (uint64_t)c->num_cus));
    k_poison_fill<<<dim3((uint32_t)blocks), dim3(256), 0, pick_stream(c, stream)>>>((uint64_t*)d_words, nwords, d_status);
    HIP_TRY(hipGetLastError());
    return LSMB_OK;
}

int lsmb_flag_signal_dev(lsmb_ctx* c, uint32_t* d_flag, uint32_t value, void* stream) {
    if (!c || !d_flag) return fail(LSMB_EINVAL, "null argument");
    if (((uintptr_t)d_flag & 3) != 0) return fail(LSMB_EINVAL, "d_flag is not 4-byte aligned");
    DevGuard g(c->dev);
    k_flag_signal<<<dim3(1), dim3(64), 0, pick_stream(c, stream)>>>(d_flag, value);
    HIP_TRY(hipGetLastError());
    return LSMB_OK;
}

int lsmb_flag_wait_dev(lsmb_ctx* c, const uint32_t* const* d_flags, const uint32_t* const* d_poison, uint32_t nflags,
                       uint32_t value, uint32_t timeout_ms, uint32_t* d_status, void* stream) {
    if (!c || !d_flags || !d_status) return fail(LSMB_EINVAL, "null argument");
    if (nflags > kMaxFlags) return fail(LSMB_EINVAL, "nflags must be at most %u", kMaxFlags);
    if (((uintptr_t)d_status & 3) != 0) return fail(LSMB_EINVAL, "d_status is not 4-byte aligned");
    FlagSet fs, ps;
    fs.n = nflags;
    ps.n = d_poison ? nflags : 0;
    for (uint32_t j = 0; j < nflags; j++) {
        if (!d_flags[j] || ((uintptr_t)d_flags[j] & 3) != 0) return fail(LSMB_EINVAL, "flag %u: null or unaligned", j);
        fs.p[j] = d_flags[j];
        if (d_poison) {
            if (!d_poison[j] || ((uintptr_t)d_poison[j] & 3) != 0)
                return fail(LSMB_EINVAL, "poison word %u: null or unaligned", j);
            ps.p[j] = d_poison[j];
        }
    }
    DevGuard g(c->dev);
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev) != hipSuccess || khz <= 0) khz = 100000;
    const uint64_t ticks = (uint64_t)timeout_ms * (uint64_t)khz;
    k_flag_wait<<<dim3(1), dim3(64), 0, pick_stream(c, stream)>>>(fs, ps, value, ticks, d_status);
    HIP_TRY(hipGetLastError());
    return LSMB_OK;
}

int lsmb_merge_status(lsmb_ctx* c, const uint32_t* d_status, void* stream, uint32_t* out2) {
    if (!c || !d_status || !out2) return fail(LSMB_EINVAL, "null argument");
    if (((uintptr_t)d_status & 3) != 0) return fail(LSMB_EINVAL, "d_status is not 4-byte aligned");
    DevGuard g(c->dev);
    const hipStream_t st = pick_stream(c, stream);
    HIP_TRY(hipMemcpyAsync(out2, d_status, 8, hipMemcpyDeviceToHost, st));  // after the stream's waits
    HIP_TRY(hipStreamSynchronize(st));
    return LSMB_OK;
}

int lsmb_multi_last_ms(lsmb_multi* m, float* out3) {
    if (!m || !out3) return fail(LSMB_EINVAL, "null argument");
    if (!m->timed) return fail(LSMB_EINVAL, "no multi-GPU build on this handle");
    float tot = 0.f, bld = 0.f;
    for (int g = 0; g < shards(m); g++) {
        DevGuard dg(m->ctx[g]->dev);
        float a = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, m->t0[g], m->t2[g]));
        HIP_TRY(hipEventElapsedTime(&b, m->t0[g], m->t1[g]));
        tot = std::max(tot, a);
        bld = std::max(bld, b);
    }
    out3[0] = tot;
    out3[1] = bld;
    out3[2] = tot - bld;
    return LSMB_OK;
}

}  // extern "C"
