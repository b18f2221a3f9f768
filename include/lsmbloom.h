/*
 * lsmbloom.h — C ABI of the MI355X-native Bloom-filter engine.
 *
 * Drop-in boundary for G1DO/Storage-Engine `src/bloom` (Rust).  The store's
 * callers — SSTableBuilder (src/sstable/builder.rs:74,93,177-182), SSTable::open
 * (src/sstable/reader.rs:78-82), SSTable::get (src/sstable/reader.rs:197) — keep
 * calling the Rust surface `crate::bloom::{BloomFilter, BloomFilterBuilder}`;
 * a thin Rust shim forwards to the entry points below.
 *
 * Conventions
 *   - Plain pointers and sizes only; all buffers are caller-owned and the
 *     library keeps no pointer after a call returns.
 *   - Return 0 (LSMB_OK) on success, a negative LSMB_E* code otherwise; the
 *     thread-local message of the last failure is lsmb_last_error().
 *   - Where the reference panics (assert!/division by zero), the ABI returns
 *     LSMB_EINVAL; where it returns Err(Error::Corruption) (deserialize), the
 *     ABI returns LSMB_ECORRUPT (src/error.rs:12).
 *   - Filter words are the reference's `bits: Vec<u64>` (src/bloom/mod.rs:24):
 *     ceil(num_bits/64) little-endian u64, bit p = word p/64, bit p%64.
 *   - Batched build entry points OR-ACCUMULATE into `words` (existing bits are
 *     kept), so a build after insert()s, or a merge of shard partials, is exact.
 *   - Batched entry points run on the GPU.  With no usable gfx950 device,
 *     lsmb_open fails with LSMB_ENODEV: there is no silent CPU fallback.  The
 *     one host path is deliberate and size-bounded: host-memory builds of at
 *     most lsmb_host_max_keys() keys (an SST flush of the reference's default
 *     1 000-key sizing, src/sstable/builder.rs:51,74) run the library's own
 *     per-key loop, where a device round trip costs more than the whole build;
 *     for those ctx may be NULL, so the store works on a host without a GPU.
 *   - Thread safety: a context may be used from one thread at a time; distinct
 *     contexts (e.g. flush + background compaction, src/compaction/scheduler.rs:37)
 *     may run concurrently.  Stateless functions are always thread safe.
 */
#ifndef LSMBLOOM_H
#define LSMBLOOM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSMB_OK 0
#define LSMB_EINVAL (-1)   /* argument the reference rejects by panicking      */
#define LSMB_ENODEV (-2)   /* no gfx950 device / HIP initialisation failed     */
#define LSMB_EHIP (-3)     /* HIP runtime or kernel launch error               */
#define LSMB_ECORRUPT (-4) /* serialized filter fails validation               */
#define LSMB_ENOMEM (-5)   /* device or pinned-host allocation failed          */

#define LSMB_ABI_VERSION 6 /* 5: sweep builds, block CRC-32; 6: fail-safe merge status words */

typedef struct lsmb_ctx lsmb_ctx; /* one GPU: stream, events, scratch arenas */

int lsmb_abi_version(void);
const char* lsmb_last_error(void);

/* ---- sizing ------------------------------------------------------------ */

/* BloomFilter::new(expected_items, false_positive_rate) sizing
 * (src/bloom/mod.rs:38-67): num_bits = max(sat_u32(ceil(n * -1.44*log2 fpr)), 64),
 * num_hashes = max(ceil(bpk * ln 2), 1).  LSMB_EINVAL where the reference
 * panics (n == 0, fpr outside (0,1); :39-43). */
int lsmb_params(uint64_t expected_items, double false_positive_rate, uint32_t* num_bits,
                uint32_t* num_hashes);

/* ceil(num_bits / 64): length of the words array (src/bloom/mod.rs:58). */
uint64_t lsmb_num_words(uint32_t num_bits);

/* ---- format (src/bloom/mod.rs:102-168) --------------------------------- */

/* 12 + 8 * ceil(num_bits/64)  (serialize, :102-115). */
uint64_t lsmb_serialized_size(uint32_t num_bits);

/* BloomFilter::serialize (:102-115): [num_hashes u32][num_bits u32]
 * [num_u64s u32][words u64...] little-endian.  out_len must be >= the size. */
int lsmb_serialize(const uint64_t* words, uint32_t num_bits, uint32_t num_hashes, uint8_t* out,
                   uint64_t out_len);

/* BloomFilter::deserialize validation (:123-153): len >= 12, num_u64s ==
 * ceil(num_bits/64), len == 12 + 8*num_u64s; else LSMB_ECORRUPT. */
int lsmb_deserialize_header(const uint8_t* data, uint64_t len, uint32_t* num_hashes,
                            uint32_t* num_bits, uint32_t* num_u64s);

/* Validates like lsmb_deserialize_header, then copies the words (:156-161). */
int lsmb_deserialize(const uint8_t* data, uint64_t len, uint64_t* words, uint64_t words_cap);

/* ---- single-key operations (BloomFilter::insert / may_contain) ---------- */

/* BloomFilter::insert (src/bloom/mod.rs:70-78) on host-resident words: one
 * key, so no device round trip (a launch costs ~10 us, the insert ~20 ns). */
int lsmb_insert(uint64_t* words, uint32_t num_bits, uint32_t num_hashes, const uint8_t* key,
                uint64_t key_len);

/* BloomFilter::may_contain (:82-94).  Returns 1 / 0, or < 0 on error. */
int lsmb_may_contain(const uint64_t* words, uint32_t num_bits, uint32_t num_hashes,
                     const uint8_t* key, uint64_t key_len);

/* Debug/test helper: the k bit positions of one key (hash_key + get_position,
 * src/bloom/mod.rs:181-197). */
int lsmb_positions(const uint8_t* key, uint64_t key_len, uint32_t num_bits, uint32_t num_hashes,
                   uint32_t* out_positions);

/* ---- GPU context --------------------------------------------------------- */

/* Opens `device` (HIP ordinal; -1 = current device).  LSMB_ENODEV if no
 * gfx950 device is usable. */
int lsmb_open(lsmb_ctx** out, int device);
void lsmb_close(lsmb_ctx* ctx);

/* Blocks until all work issued on the context's stream has finished. */
int lsmb_sync(lsmb_ctx* ctx);

/* ---- batched build (BloomFilterBuilder::add_key loop + build) ------------ */
/* Host-memory entry points: the keys go up in chunks through two device
 * staging slots (chunk i+1's H2D overlaps chunk i's kernels), the build runs on
 * the GPU, the words come back (OR-accumulated into `words`).  Synchronous.
 * n <= lsmb_host_max_keys(): the library's host loop builds the same bits with
 * no device round trip, and ctx may be NULL (above it, NULL is LSMB_EINVAL). */

/* Size threshold of the host path (default 2048 keys, env LSMB_HOST_MAX_KEYS;
 * 0 sends every build to the GPU).  The bits never depend on it. */
uint64_t lsmb_host_max_keys(void);
void lsmb_set_host_max_keys(uint64_t n);

/* n keys of key_len bytes each, packed back to back (key i at keys + i*key_len). */
int lsmb_build_fixed(lsmb_ctx* ctx, const uint8_t* keys, uint32_t key_len, uint64_t n,
                     uint32_t num_bits, uint32_t num_hashes, uint64_t* words);

/* n variable-length keys: key i = data[offsets[i] .. offsets[i+1]). */
int lsmb_build_var(lsmb_ctx* ctx, const uint8_t* data, const uint64_t* offsets, uint64_t n,
                   uint32_t num_bits, uint32_t num_hashes, uint64_t* words);

/* The SSTable bloom block in one call: replaces
 *     let bloom = self.bloom_builder.build();   let bloom_data = bloom.serialize();
 * of SSTableBuilder::finish (src/sstable/builder.rs:177-179).  Builds a fresh
 * filter (BloomFilter::new(..) then insert of every key, src/bloom/mod.rs:38-78)
 * from n host-memory keys — fixed-length (offsets == NULL, key i at
 * data + i*key_len) or variable-length (key i = data[offsets[i]..offsets[i+1])) —
 * and writes exactly the bytes BloomFilter::serialize returns
 * (src/bloom/mod.rs:102-115) into block[0 .. lsmb_serialized_size(num_bits)).
 * The words go device -> block directly (no host word array, no serialize
 * copy); the key H2D is chunked and overlapped with the build kernels.
 * n == 0 gives the empty filter's block.  block_len < the size: LSMB_EINVAL. */
int lsmb_build_block(lsmb_ctx* ctx, const uint8_t* data, const uint64_t* offsets, uint32_t key_len,
                     uint64_t n, uint32_t num_bits, uint32_t num_hashes, uint8_t* block,
                     uint64_t block_len);

/* ---- streaming ingestion (the flush / compaction add_key loop) ----------- */
/* The store's flush walks the frozen memtable and adds every key
 * (src/db/mod.rs:379-383 -> SSTableBuilder::add -> BloomFilterBuilder::add_key,
 * src/sstable/builder.rs:93); compaction does the same over its merged
 * entries (src/compaction/scheduler.rs:113-125,152-158).  An lsmb_stream takes
 * those keys one at a time while the walk is still going: each add is a copy
 * into pinned staging, and every full staging chunk (LSMB_STREAM_CHUNK_MB,
 * default 128) is uploaded and built asynchronously while the caller keeps
 * adding into the other chunk.  finish writes the serialized bloom block (or
 * the words) of BloomFilter::new + insert of every added key.  A run of at
 * most lsmb_host_max_keys() keys never touches the device (host loop at
 * finish); with ctx == NULL the stream is host-only and finish of a larger
 * run is LSMB_EINVAL.  One stream per thread; reusable after finish
 * (lsmb_stream_reset for another filter size). */
typedef struct lsmb_stream lsmb_stream;

int lsmb_stream_open(lsmb_ctx* ctx, uint32_t num_bits, uint32_t num_hashes, lsmb_stream** out);
int lsmb_stream_reset(lsmb_stream* s, uint32_t num_bits, uint32_t num_hashes);
void lsmb_stream_close(lsmb_stream* s);

/* BloomFilterBuilder::add_key (src/bloom/builder.rs:21-23): appends one key. */
int lsmb_stream_add(lsmb_stream* s, const uint8_t* key, uint64_t key_len);

/* Appends n keys: key i = data[offsets[i] .. offsets[i+1]). */
int lsmb_stream_add_batch(lsmb_stream* s, const uint8_t* data, const uint64_t* offsets, uint64_t n);

/* Keys added since open / the last finish. */
uint64_t lsmb_stream_count(const lsmb_stream* s);

/* Finishes the filter: the bytes BloomFilter::serialize returns
 * (src/bloom/mod.rs:102-115) into block[0 .. lsmb_serialized_size(num_bits)),
 * or the ceil(num_bits/64) words.  Synchronous; the stream then starts a new,
 * empty filter of the same size. */
int lsmb_stream_finish_block(lsmb_stream* s, uint8_t* block, uint64_t block_len);
int lsmb_stream_finish_words(lsmb_stream* s, uint64_t* words);

/* ---- batched probe (may_contain over a batch of keys x filters) --------- */
/* For key i and filter f: bit (f % 8) of out_mask[i * ceil(nfilt/8) + f / 8]
 * = may_contain(filter f, key i), exactly what SSTable::get's bloom check
 * (src/sstable/reader.rs:197) answers for that SSTable.  offsets == NULL
 * selects fixed-length keys of key_len bytes.  nfilt <= 64. */
int lsmb_probe(lsmb_ctx* ctx, const uint64_t* const* filt_words, const uint32_t* filt_bits,
               const uint32_t* filt_hashes, uint32_t nfilt, const uint8_t* data,
               const uint64_t* offsets, uint32_t key_len, uint64_t n, uint8_t* out_mask);

/* ---- device-resident entry points ---------------------------------------- */
/* All pointers are device pointers (hipMalloc).  `stream` is a hipStream_t
 * (NULL = the context's own stream).  Asynchronous: the call returns after
 * enqueueing; synchronise on the stream before reading results. */

int lsmb_build_fixed_dev(lsmb_ctx* ctx, const void* d_keys, uint32_t key_len, uint64_t n,
                         uint32_t num_bits, uint32_t num_hashes, void* d_words, void* stream);

int lsmb_build_var_dev(lsmb_ctx* ctx, const void* d_data, const void* d_offsets, uint64_t n,
                       uint32_t num_bits, uint32_t num_hashes, void* d_words, void* stream);

/* BloomFilterBuilder::{new, add_key per key, build} (src/bloom/builder.rs:14-28) into device words:
 * BloomFilter::new (src/bloom/mod.rs:38-67) + insert of every key.  Unlike the
 * entry points above, `d_words` is OUTPUT-ONLY — its old contents are ignored,
 * every word of the filter is written — so the build needs no zeroing pass and
 * never reads the old words.  n == 0 or num_hashes == 0 writes all-zero words.
 * Memory: a partitioned k = 7 build also allocates, once per context and kept
 * until lsmb_close, an overflow bitmap as large as the filter (C2: 120 MB; the
 * 2^32-1-bit C5 filter: 512 MiB), 4 bytes per 2^20 filter bits of unit marks,
 * and 64 KiB of overflow lists per pass A workgroup per sweep (C2 and C5: 32
 * MiB).  These are outside LSMB_WORKSPACE_MB, which bounds only the partition
 * regions (the key chunk size follows from it). */
int lsmb_build_fixed_dev_new(lsmb_ctx* ctx, const void* d_keys, uint32_t key_len, uint64_t n,
                             uint32_t num_bits, uint32_t num_hashes, void* d_words, void* stream);
int lsmb_build_var_dev_new(lsmb_ctx* ctx, const void* d_data, const void* d_offsets, uint64_t n,
                           uint32_t num_bits, uint32_t num_hashes, void* d_words, void* stream);

/* A partitioned build (filters above a few MiB) runs in sweeps: each re-reads
 * the keys and keeps the positions of its own range of the filter (C5's
 * 2^32-1-bit filter: 2 sweeps of 256 MiB).  lsmb_build_sweeps gives their
 * number (1 for every other strategy), lsmb_sweep_words the word range
 * [word_lo, word_hi) whose bits sweep s completes, and
 * lsmb_build_fixed_dev_sweep builds just that sweep (OR-accumulate; running
 * every sweep == lsmb_build_fixed_dev).  A sharded build can then merge sweep
 * s's word range across GPUs while sweep s+1 builds. */
int lsmb_build_sweeps(uint32_t num_bits, uint32_t num_hashes, uint64_t n);
int lsmb_sweep_words(uint32_t num_bits, uint32_t num_hashes, uint64_t n, int sweep, uint64_t* word_lo,
                     uint64_t* word_hi);
int lsmb_build_fixed_dev_sweep(lsmb_ctx* ctx, const void* d_keys, uint32_t key_len, uint64_t n,
                               uint32_t num_bits, uint32_t num_hashes, void* d_words, int sweep, void* stream);
/* Sweep s of lsmb_build_fixed_dev_new: writes every word of sweep s's range
 * [word_lo, word_hi) (output-only there), no other word.  Running every sweep
 * == lsmb_build_fixed_dev_new. */
int lsmb_build_fixed_dev_sweep_new(lsmb_ctx* ctx, const void* d_keys, uint32_t key_len, uint64_t n,
                                   uint32_t num_bits, uint32_t num_hashes, void* d_words, int sweep, void* stream);

/* CRC-32 of bloom blocks (optional checksum; the reference's
 * bloom block has none).  The same CRC as crc32fast::hash / zlib.crc32, which
 * the store already uses for WAL records and the manifest
 * (src/wal/record.rs:96,122, src/manifest/mod.rs:5).
 *   lsmb_crc32          host bytes, appended to crc (0 to start)
 *   lsmb_crc32_combine  CRC(A||B) from CRC(A), CRC(B), |B|
 *   lsmb_crc32_dev      device bytes (parallel CRC + combine), appended to crc
 *   lsmb_build_block_crc  lsmb_build_block + the block's CRC-32, the words'
 *                         part computed on the device copy before the D2H
 *   lsmb_fset_add_crc   lsmb_fset_add that checks the block's CRC-32 on the
 *                       copy in HBM: mismatch -> LSMB_ECORRUPT, slot not added */
uint32_t lsmb_crc32(uint32_t crc, const uint8_t* data, uint64_t len);
uint32_t lsmb_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
int lsmb_crc32_dev(lsmb_ctx* ctx, uint32_t crc, const void* d_data, uint64_t len, uint32_t* out, void* stream);
int lsmb_build_block_crc(lsmb_ctx* ctx, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                         uint32_t num_bits, uint32_t num_hashes, uint8_t* block, uint64_t block_len, uint32_t* crc);

/* d_filt_words: host array of nfilt DEVICE pointers. */
int lsmb_probe_dev(lsmb_ctx* ctx, const void* const* d_filt_words, const uint32_t* filt_bits,
                   const uint32_t* filt_hashes, uint32_t nfilt, const void* d_data,
                   const void* d_offsets, uint32_t key_len, uint64_t n, void* d_out_mask,
                   void* stream);

/* OR-reduce: d_dst[i] |= d_src[j*stride_words + i] for j < nsrc, i < nwords.
 * The merge step of a sharded build (partial filters -> one filter). */
int lsmb_or_reduce_dev(lsmb_ctx* ctx, void* d_dst, const void* d_src, uint64_t nwords,
                       uint32_t nsrc, uint64_t stride_words, void* stream);

/* Synthetic workload generators, device-side:
 * key16(seed, i) = LE64(splitmix64(seed+2i)) || LE64(splitmix64(seed+2i+1)),
 * for i in [first, first+n). */
int lsmb_gen_key16_dev(lsmb_ctx* ctx, uint64_t seed, uint64_t first, uint64_t n, void* d_keys,
                       void* stream);

/* u64 stream: d_out[j] = mod ? add + splitmix64(seed+first+j) % mod
 *                            : splitmix64(seed+first+j), j in [0, n).
 * The C4 var-len workload: key lengths (seed 0x5EED0003, mod 249, add 8) and
 * the packed key bytes (seed 0x5EED0004, mod 0, LE words). */
int lsmb_gen_splitmix_dev(lsmb_ctx* ctx, uint64_t seed, uint64_t first, uint64_t n, uint32_t mod,
                          uint32_t add, void* d_out, void* stream);

/* ---- one process, several GPUs (sharded build) -------------------------- */
/* When one flush / compaction run is large (src/db/mod.rs:377-383,
 * src/compaction/scheduler.rs:150-158, both feeding SSTableBuilder::add,
 * src/sstable/builder.rs:93), lsmb_multi splits its keys into G contiguous
 * shards, builds a full-size partial filter per shard on its own GPU and merges
 * the partials with a bitwise-OR reduce-scatter done by peer loads over xGMI.
 * OR is associative, commutative and idempotent: the merged words equal a
 * single-device build of all the keys, bit for bit.  Devices may repeat (the
 * shards then share a GPU).  Used from one thread at a time. */
typedef struct lsmb_multi lsmb_multi;

/* devices: ndev HIP ordinals (NULL = 0..ndev-1), 1 <= ndev <= 16.  Enables
 * peer access between every pair of distinct devices (LSMB_ENODEV if a pair
 * has no peer path). */
int lsmb_multi_open(lsmb_multi** out, const int* devices, int ndev);
void lsmb_multi_close(lsmb_multi* m);
int lsmb_multi_size(const lsmb_multi* m);

/* Shard g's single-GPU context (its device, stream and scratch), e.g. to place
 * device buffers or run other entry points on that GPU. */
lsmb_ctx* lsmb_multi_ctx(lsmb_multi* m, int shard);

/* Device-resident sharded build: shard g's n[g] keys of key_len bytes at
 * d_keys[g] and its words d_words[g] live on shard g's device.  Every shard
 * builds into its own words (OR-accumulate), then reduce-scatter + all-gather:
 * on return every d_words[g] holds the merged filter.  Synchronous. */
int lsmb_multi_build_fixed_dev(lsmb_multi* m, const void* const* d_keys, const uint64_t* n, uint32_t key_len,
                               uint32_t num_bits, uint32_t num_hashes, void* const* d_words);

/* lsmb_build_block over G GPUs: the n host-memory keys (fixed-length, or
 * var-length with offsets) are split into G contiguous shards; each GPU
 * uploads and builds its shard (G PCIe links in parallel), the partials are
 * OR-reduce-scattered over xGMI, and each GPU copies its merged word slice
 * into the block.  Writes exactly BloomFilter::serialize's bytes. */
int lsmb_multi_build_block(lsmb_multi* m, const uint8_t* data, const uint64_t* offsets, uint32_t key_len,
                           uint64_t n, uint32_t num_bits, uint32_t num_hashes, uint8_t* block,
                           uint64_t block_len);

/* Timing of the last multi build, ms: [0] total (slowest shard), [1] build
 * (slowest shard), [2] merge = [0] - [1]. */
int lsmb_multi_last_ms(lsmb_multi* m, float* out3);

/* ---- one process per GPU: cross-process peer-load merge ------------------- */
/* The same OR merge between processes (one per GPU, e.g. torch.distributed
 * ranks), without a collective library: every rank exports the device
 * allocation holding its partial words, maps the other ranks' allocations
 * (over xGMI when they sit on other GPUs of the node; the same HBM when they
 * share one), and merges with peer loads: rank g ORs word-slice g of every
 * partial into its own words (lsmb_or_gather_dev with all G sources), then
 * copies every other merged slice from its owner (one source each).  The
 * caller orders the ranks between the phases: a host barrier after each
 * rank's stream has finished, or the device flags below.  Replaces what RCCL cannot do in one call (it
 * has no bitwise-OR reduction) for the sharded flush / compaction of
 * src/db/mod.rs:377-383 and src/compaction/scheduler.rs:150-158. */
#define LSMB_IPC_HANDLE_BYTES 64

/* Handle of the device allocation holding d_ptr (hipIpcGetMemHandle) and
 * d_ptr's byte offset in it. */
int lsmb_ipc_export(const void* d_ptr, uint8_t* handle, uint64_t* offset);

/* Maps another process's allocation into this context's device
 * (hipIpcOpenMemHandle, peer access enabled lazily); *d_base = its first
 * byte here.  A handle exported by this same process is LSMB_EINVAL. */
int lsmb_ipc_import(lsmb_ctx* ctx, const uint8_t* handle, void** d_base);

/* Unmaps an allocation lsmb_ipc_import mapped (d_base as returned). */
int lsmb_ipc_close(lsmb_ctx* ctx, void* d_base);

/* Merge status words (round 6): LSMB_MERGE_STATUS_WORDS u32 in device memory,
 * zero when the merge is set up, owned by one merge (one per IpcMerge):
 *   [0] poison: set (sticky) once one of the merge's phase waits timed out or
 *       saw another rank's poison;
 *   [1] the merge's phase waits that timed out.
 * A poisoned merge never reads its peers' words again and leaves every range
 * it merges all-ones: all-ones is a superset of every partial, so the filter
 * can answer "maybe" too often but never "no" for a key that was added (a
 * false negative would make DB::get skip the SST holding the key,
 * src/sstable/reader.rs:196-199, src/db/mod.rs:243-267).  The caller learns
 * of it at its next sync point (lsmb_merge_status) and must not trust the
 * filter as exact.  The status words live in the flag allocation the peers
 * map, so that a rank's poison is visible to every peer's waits. */
#define LSMB_MERGE_STATUS_WORDS 2

/* d_dst[i] = OR over j < nsrc of d_srcs[j][i], i < nwords (u64 words; any
 * source may be d_dst itself, or mapped peer memory).  Asynchronous on
 * `stream`.  nsrc == 1 is a copy; 1 <= nsrc <= 16.  d_status (NULL: none):
 * when the merge is poisoned at kernel time, d_dst[0, nwords) = all-ones and
 * no source is read. */
int lsmb_or_gather_dev(lsmb_ctx* ctx, void* d_dst, const void* const* d_srcs, uint32_t nsrc, uint64_t nwords,
                       const uint32_t* d_status, void* stream);

/* The merge's all-gather in one call: for every slice r < nsrc with
 * d_srcs[r] != NULL, d_dst[w] = d_srcs[r][w] for w in [r slice_words,
 * min((r+1) slice_words, nwords)) (u64 words; a NULL source leaves its slice
 * alone, e.g. the caller's own).  One kernel streams every slice at once, so
 * every peer link is busy.  The sources (mapped peer memory, or other local
 * buffers) must not overlap d_dst.  Asynchronous on `stream`.  d_status as
 * above: poisoned, those slices are written all-ones. */
int lsmb_copy_slices_dev(lsmb_ctx* ctx, void* d_dst, const void* const* d_srcs, uint32_t nsrc, uint64_t slice_words,
                         uint64_t nwords, const uint32_t* d_status, void* stream);

/* The merge's last step: if the merge is poisoned once everything before this
 * on `stream` has run, d_words[0, nwords) = all-ones; otherwise nothing. */
int lsmb_poison_fill_dev(lsmb_ctx* ctx, void* d_words, uint64_t nwords, const uint32_t* d_status, void* stream);

/* Device-ordered phases for the merge above, so that no host waits inside it:
 * a flag is a u32 epoch counter in device memory (this process's own, or a
 * peer's mapped with lsmb_ipc_import).  The merge of epoch e on `stream` is
 *   signal(own flag[0], e); wait(every rank's flag[0] >= e)   partials final
 *   or_gather (reduce-scatter);  signal(flag[1], e); wait(all flag[1] >= e)
 *   copy_slices (all-gather); signal(flag[2], e); wait(all flag[2] >= e)
 *   poison_fill
 * (lsmbloom.dist.IpcMerge, lsmbloom.dist.merge_schedule).  All enqueue and
 * return at once. */

/* After everything before it on `stream`: a system-scope release store of
 * `value` into *d_flag. */
int lsmb_flag_signal_dev(lsmb_ctx* ctx, uint32_t* d_flag, uint32_t value, void* stream);

/* Later work on `stream` waits until every d_flags[j] >= value (epoch compare,
 * wrap-safe), j < nflags <= 64.  d_poison[j] (or NULL) = rank j's poison word
 * (its status word [0]; the caller's own among them).  The wait ends early,
 * and poisons this merge (d_status[0] = 1), when any poison word is set, also
 * when one is set after the flags were met; a flag still short after
 * timeout_ms counts a timeout (d_status[1] += 1), poisons the merge and ends
 * the wait: a dead peer can never hang the queue, and never yields a filter
 * with missing bits. */
int lsmb_flag_wait_dev(lsmb_ctx* ctx, const uint32_t* const* d_flags, const uint32_t* const* d_poison, uint32_t nflags,
                       uint32_t value, uint32_t timeout_ms, uint32_t* d_status, void* stream);

/* The merge's sync point: waits for `stream`, then out2 = {poison, timeouts}
 * (the status words above). */
int lsmb_merge_status(lsmb_ctx* ctx, const uint32_t* d_status, void* stream, uint32_t* out2);

/* ---- device-resident filter sets (multi-get pre-check) --------------------- */
/* An lsmb_fset keeps up to 64 SSTable filters resident in device memory, each
 * with its table's key range [min_key, max_key] (SSTable meta,
 * src/sstable/reader.rs:192).  A probe answers, per key and per filter, the two
 * checks SSTable::get makes before it touches the index (reader.rs:192-199):
 *     min_key <= key <= max_key   (byte-wise lexicographic, as Rust's [u8] Ord)
 *     && may_contain(filter, key)
 * for a whole batch of keys, so DB::get (src/db/mod.rs:243-267), which today
 * re-opens and re-deserializes every SSTable per lookup (mod.rs:245,259), can
 * keep its filters on the GPU and read only the tables a key may be in.
 * A set belongs to one context and is used from one thread at a time. */
typedef struct lsmb_fset lsmb_fset;

int lsmb_fset_open(lsmb_ctx* ctx, lsmb_fset** out);
void lsmb_fset_close(lsmb_fset* fs);

/* Adds a filter from its serialized bloom block (the bytes BloomFilter::serialize
 * wrote, src/bloom/mod.rs:102-115), validated exactly as BloomFilter::deserialize
 * (mod.rs:123-168; LSMB_ECORRUPT) and copied straight into device memory.
 * Returns the filter's slot (0..63, bit `slot` of the probe mask) or < 0. */
int lsmb_fset_add(lsmb_fset* fs, const uint8_t* block, uint64_t len, const uint8_t* min_key,
                  uint64_t min_len, const uint8_t* max_key, uint64_t max_len);

/* lsmb_fset_add that also checks the block's CRC-32 (lsmb_crc32 /
 * crc32fast::hash of all `len` bytes) on the copy in device memory. */
int lsmb_fset_add_crc(lsmb_fset* fs, const uint8_t* block, uint64_t len, uint32_t crc, const uint8_t* min_key,
                      uint64_t min_len, const uint8_t* max_key, uint64_t max_len);

/* Same from in-memory filter words (ceil(num_bits/64) LE u64). */
int lsmb_fset_add_words(lsmb_fset* fs, const uint64_t* words, uint32_t num_bits, uint32_t num_hashes,
                        const uint8_t* min_key, uint64_t min_len, const uint8_t* max_key,
                        uint64_t max_len);

/* Drops a filter (e.g. its table was compacted away); the slot is re-used. */
int lsmb_fset_remove(lsmb_fset* fs, int slot);

/* Bit s set = slot s holds a filter. */
uint64_t lsmb_fset_live_mask(const lsmb_fset* fs);

/* out_mask[i] bit s = (min_s <= key i <= max_s) && may_contain(filter s, key i).
 * offsets == NULL selects fixed-length keys of key_len bytes.  Synchronous. */
int lsmb_fset_probe(lsmb_fset* fs, const uint8_t* data, const uint64_t* offsets, uint32_t key_len,
                    uint64_t n, uint64_t* out_mask);

/* Device-memory keys and output (u64 per key); asynchronous on `stream`. */
int lsmb_fset_probe_dev(lsmb_fset* fs, const void* d_data, const void* d_offsets, uint32_t key_len,
                        uint64_t n, void* d_out_mask, void* stream);

/* lsmb_fset_probe_dev with answer rows of row_bytes = 1, 2, 4 or 8 bytes: row i
 * is the u64 mask's low row_bytes bytes (LE), so a set whose live slots are
 * all below 8 * row_bytes (e.g. 8 per-level tables in 1 byte) writes 1/8 of
 * the u64 rows' bytes.  A live slot at or above 8 * row_bytes is LSMB_EINVAL. */
int lsmb_fset_probe_dev_rows(lsmb_fset* fs, const void* d_data, const void* d_offsets, uint32_t key_len, uint64_t n,
                             void* d_out, uint32_t row_bytes, void* stream);

/* ---- introspection ------------------------------------------------------- */

/* Name of the device build strategy the dispatcher picks for (num_bits, k, n):
 * "lds", "tiled", "partition", "atomic" (for tests and bench reporting).
 * Host-memory builds of n <= lsmb_host_max_keys() keys run on the host instead.
 * Measurement switches read at build time: LSMB_FORCE_STRATEGY=atomic,
 * LSMB_SWEEP_PER=1/2 (pass A keys per lane), LSMB_TILED_NO_PREHASH=1,
 * LSMB_H2D_CHUNK_MB, LSMB_WORKSPACE_MB.  The filter bits never depend on them. */
const char* lsmb_build_strategy(uint32_t num_bits, uint32_t num_hashes, uint64_t n);

/* Timing of the last device build on this context, in milliseconds, per phase
 * (HIP events on the build stream): [0] total, [1] pass A (hash + bin),
 * [2] pass B (apply).  Waits for the timed build to finish (on whatever
 * stream it was issued). */
int lsmb_last_build_ms(lsmb_ctx* ctx, float* out3);

/* Per-build HIP events behind lsmb_last_build_ms: on (1, the default) or off
 * (0: a build issues only its kernels, no timing markers between them). */
int lsmb_set_timing(lsmb_ctx* ctx, int enable);

#ifdef __cplusplus
}
#endif

#endif /* LSMBLOOM_H */
