"""lsmbloom — Python binding of the MI355X Bloom engine's C ABI (include/lsmbloom.h).

Mirrors the reference's Rust surface `crate::bloom` (G1DO/Storage-Engine
src/bloom/mod.rs, src/bloom/builder.rs) so tests read like the reference's own:

    bf = BloomFilter.new(100, 0.01)      # BloomFilter::new            mod.rs:38-67
    bf.insert(b"hello")                  # BloomFilter::insert         mod.rs:70-78
    bf.may_contain(b"hello")             # BloomFilter::may_contain    mod.rs:82-94
    bf.serialize() / BloomFilter.deserialize(b)                      # mod.rs:102-168
    b = BloomFilterBuilder.new(n, fpr); b.add_key(k); bf = b.build()  # builder.rs:14-28

Batched work (BloomFilterBuilder.build, probe_batch) runs on the GPU through
the C ABI; it raises if the HIP library or a gfx950 device is missing — there
is no CPU fallback.  The one host path is the library's own, size-bounded:
builds of at most host_max_keys() keys (an SST flush at the reference's
default 1 000-key sizing) run its native per-key loop and need no GPU.
Device-resident entry points take torch tensors.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSMB_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "liblsmbloom.so")  # LSMB_LIB: instrumented builds (tools/)

LSMB_OK = 0
LSMB_EINVAL = -1
LSMB_ENODEV = -2
LSMB_EHIP = -3
LSMB_ECORRUPT = -4
LSMB_ENOMEM = -5

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p

# name -> (restype, argtypes); the exact export list of include/lsmbloom.h
SIGNATURES = {
    "lsmb_abi_version": (ctypes.c_int, []),
    "lsmb_last_error": (ctypes.c_char_p, []),
    "lsmb_params": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_double, u32p, u32p]),
    "lsmb_num_words": (ctypes.c_uint64, [ctypes.c_uint32]),
    "lsmb_serialized_size": (ctypes.c_uint64, [ctypes.c_uint32]),
    "lsmb_serialize": (ctypes.c_int, [u64p, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint64]),
    "lsmb_deserialize_header": (ctypes.c_int, [u8p, ctypes.c_uint64, u32p, u32p, u32p]),
    "lsmb_deserialize": (ctypes.c_int, [u8p, ctypes.c_uint64, u64p, ctypes.c_uint64]),
    "lsmb_insert": (ctypes.c_int, [u64p, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint64]),
    "lsmb_may_contain": (ctypes.c_int, [u64p, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint64]),
    "lsmb_positions": (ctypes.c_int, [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u32p]),
    "lsmb_open": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int]),
    "lsmb_close": (None, [vp]),
    "lsmb_sync": (ctypes.c_int, [vp]),
    "lsmb_build_fixed": (ctypes.c_int, [vp, u8p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_uint32, u64p]),
    "lsmb_build_var": (ctypes.c_int, [vp, u8p, u64p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u64p]),
    "lsmb_build_block": (ctypes.c_int, [vp, u8p, u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_uint32, u8p, ctypes.c_uint64]),
    "lsmb_build_block_crc": (ctypes.c_int, [vp, u8p, u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint32, u8p, ctypes.c_uint64, u32p]),
    "lsmb_crc32": (ctypes.c_uint32, [ctypes.c_uint32, u8p, ctypes.c_uint64]),
    "lsmb_crc32_combine": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "lsmb_crc32_dev": (ctypes.c_int, [vp, ctypes.c_uint32, vp, ctypes.c_uint64, u32p, vp]),
    "lsmb_fset_add_crc": (ctypes.c_int, [vp, u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_uint64, u8p,
                                         ctypes.c_uint64]),
    "lsmb_probe": (ctypes.c_int, [vp, ctypes.POINTER(u64p), u32p, u32p, ctypes.c_uint32, u8p, u64p,
                                  ctypes.c_uint32, ctypes.c_uint64, u8p]),
    "lsmb_build_fixed_dev": (ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint32, vp, vp]),
    "lsmb_build_var_dev": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                          vp, vp]),
    "lsmb_build_fixed_dev_new": (ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.c_uint32, vp, vp]),
    "lsmb_build_var_dev_new": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                              vp, vp]),
    "lsmb_probe_dev": (ctypes.c_int, [vp, ctypes.POINTER(vp), u32p, u32p, ctypes.c_uint32, vp, vp,
                                      ctypes.c_uint32, ctypes.c_uint64, vp, vp]),
    "lsmb_or_reduce_dev": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, vp]),
    "lsmb_gen_key16_dev": (ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, vp, vp]),
    "lsmb_gen_splitmix_dev": (ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint32, vp, vp]),
    "lsmb_fset_open": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
    "lsmb_fset_close": (None, [vp]),
    "lsmb_fset_add": (ctypes.c_int, [vp, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64]),
    "lsmb_fset_add_words": (ctypes.c_int, [vp, u64p, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint64, u8p,
                                           ctypes.c_uint64]),
    "lsmb_fset_remove": (ctypes.c_int, [vp, ctypes.c_int]),
    "lsmb_fset_live_mask": (ctypes.c_uint64, [vp]),
    "lsmb_fset_probe": (ctypes.c_int, [vp, u8p, u64p, ctypes.c_uint32, ctypes.c_uint64, u64p]),
    "lsmb_fset_probe_dev": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp, vp]),
    "lsmb_fset_probe_dev_rows": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp, ctypes.c_uint32, vp]),
    "lsmb_build_strategy": (ctypes.c_char_p, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "lsmb_host_max_keys": (ctypes.c_uint64, []),
    "lsmb_build_sweeps": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "lsmb_sweep_words": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, u64p, u64p]),
    "lsmb_build_fixed_dev_sweep": (ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                                  ctypes.c_uint32, vp, ctypes.c_int, vp]),
    "lsmb_build_fixed_dev_sweep_new": (ctypes.c_int, [vp, vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                                      ctypes.c_uint32, vp, ctypes.c_int, vp]),
    "lsmb_set_host_max_keys": (None, [ctypes.c_uint64]),
    "lsmb_multi_open": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "lsmb_multi_close": (None, [vp]),
    "lsmb_multi_size": (ctypes.c_int, [vp]),
    "lsmb_multi_ctx": (vp, [vp, ctypes.c_int]),
    "lsmb_multi_build_fixed_dev": (ctypes.c_int, [vp, ctypes.POINTER(vp), u64p, ctypes.c_uint32, ctypes.c_uint32,
                                                  ctypes.c_uint32, ctypes.POINTER(vp)]),
    "lsmb_multi_build_block": (ctypes.c_int, [vp, u8p, u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_uint32, u8p, ctypes.c_uint64]),
    "lsmb_multi_last_ms": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_float)]),
    "lsmb_ipc_export": (ctypes.c_int, [vp, u8p, u64p]),
    "lsmb_ipc_import": (ctypes.c_int, [vp, u8p, ctypes.POINTER(vp)]),
    "lsmb_ipc_close": (ctypes.c_int, [vp, vp]),
    "lsmb_or_gather_dev": (ctypes.c_int, [vp, vp, ctypes.POINTER(vp), ctypes.c_uint32, ctypes.c_uint64, vp, vp]),
    "lsmb_copy_slices_dev": (ctypes.c_int, [vp, vp, ctypes.POINTER(vp), ctypes.c_uint32, ctypes.c_uint64,
                                            ctypes.c_uint64, vp, vp]),
    "lsmb_poison_fill_dev": (ctypes.c_int, [vp, vp, ctypes.c_uint64, vp, vp]),
    "lsmb_flag_signal_dev": (ctypes.c_int, [vp, vp, ctypes.c_uint32, vp]),
    "lsmb_flag_wait_dev": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, vp, vp]),
    "lsmb_merge_status": (ctypes.c_int, [vp, vp, vp, u32p]),
    "lsmb_stream_open": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(vp)]),
    "lsmb_stream_reset": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32]),
    "lsmb_stream_close": (None, [vp]),
    "lsmb_stream_add": (ctypes.c_int, [vp, u8p, ctypes.c_uint64]),
    "lsmb_stream_add_batch": (ctypes.c_int, [vp, u8p, u64p, ctypes.c_uint64]),
    "lsmb_stream_count": (ctypes.c_uint64, [vp]),
    "lsmb_stream_finish_block": (ctypes.c_int, [vp, u8p, ctypes.c_uint64]),
    "lsmb_stream_finish_words": (ctypes.c_int, [vp, u64p]),
    "lsmb_last_build_ms": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_float)]),
    "lsmb_set_timing": (ctypes.c_int, [vp, ctypes.c_int]),
}

_lib = None


class LsmbError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("lsmb error %d: %s" % (code, msg))
        self.code = code


class Corruption(LsmbError):
    """Error::Corruption(String) of the reference (src/error.rs:12)."""


def lib():
    """Loads liblsmbloom.so; raises if the HIP library was not built (no fallback)."""
    global _lib
    if _lib is None:
        # Load torch's HIP runtime FIRST when torch is present: liblsmbloom.so
        # needs libamdhip64.so.7, and torch ships its own copy under the same
        # SONAME, so the loader then binds us to torch's runtime.  One runtime
        # per process means torch tensors, torch streams and RCCL share device
        # state with our kernels (loading ours first would start a second
        # runtime and break torch's CUDA init).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError("liblsmbloom.so not built (%s); run `make -C storage-engine_amd`" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("LSMB_LIB") and not hasattr(L, name):
                continue  # an older library for an A/B run (tools/): entry points it predates stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc < 0:
        msg = lib().lsmb_last_error().decode(errors="replace")
        if rc == LSMB_ECORRUPT:
            raise Corruption(rc, msg)
        if rc == LSMB_EINVAL:
            raise ValueError(msg)
        raise LsmbError(rc, msg)
    return rc


def _p(a, t):
    return a.ctypes.data_as(t)


def _key(b):
    b = bytes(b)
    a = np.frombuffer(b + b"\0", dtype=np.uint8)
    return a, len(b)


def params(expected_items, false_positive_rate):
    """BloomFilter::new sizing -> (num_bits, num_hashes); ValueError where the reference panics."""
    nb, k = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().lsmb_params(int(expected_items), float(false_positive_rate), ctypes.byref(nb), ctypes.byref(k)))
    return nb.value, k.value


def ipc_export(t):
    """(handle bytes, byte offset) of the device allocation holding tensor t's
    storage (lsmb_ipc_export), for another process's Context.ipc_import."""
    h = np.zeros(64, dtype=np.uint8)
    off = ctypes.c_uint64()
    _check(lib().lsmb_ipc_export(vp(t.data_ptr()), _p(h, u8p), ctypes.byref(off)))
    return h.tobytes(), off.value


def num_words(num_bits):
    return int(lib().lsmb_num_words(num_bits))


def serialized_size(num_bits):
    return int(lib().lsmb_serialized_size(num_bits))


def positions(key, num_bits, k):
    a, n = _key(key)
    out = np.zeros(max(k, 1), dtype=np.uint32)
    _check(lib().lsmb_positions(_p(a, u8p), n, num_bits, k, _p(out, u32p)))
    return [int(x) for x in out[:k]]


# ------------------------------------------------------------------ GPU context
class Context:
    """One GPU: stream + scratch arenas (lsmb_ctx).  Raises if no gfx950 device."""

    def __init__(self, device=-1):
        h = vp()
        _check(lib().lsmb_open(ctypes.byref(h), int(device)))
        self.h = h

    def close(self):
        if self.h:
            lib().lsmb_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        _check(lib().lsmb_sync(self.h))

    # host-memory entry points -------------------------------------------------
    def build_fixed(self, keys, key_len, num_bits, k, words=None):
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = keys.size // key_len if key_len else 0
        if words is None:
            words = np.zeros(num_words(num_bits), dtype=np.uint64)
        if keys.size == 0:
            keys = np.zeros(1, np.uint8)
        _check(lib().lsmb_build_fixed(self.h, _p(keys, u8p), key_len, n, num_bits, k, _p(words, u64p)))
        return words

    def build_var(self, data, offsets, num_bits, k, words=None):
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if words is None:
            words = np.zeros(num_words(num_bits), dtype=np.uint64)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        _check(lib().lsmb_build_var(self.h, _p(data, u8p), _p(offsets, u64p), offsets.size - 1, num_bits, k,
                                    _p(words, u64p)))
        return words

    def build_block(self, data, num_bits, k, offsets=None, key_len=0, out=None):
        """The serialized bloom block (BloomFilter::serialize of a fresh filter over
        the keys, src/bloom/mod.rs:102-115) in one call: lsmb_build_block.  Keys are
        fixed-length (key_len) or var-length (offsets, n+1 u64).  `out` may be a
        preallocated uint8 array (e.g. the SST write buffer); returns the array."""
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n = offsets.size - 1
            op = _p(offsets, u64p)
        else:
            n = data.size // key_len if key_len else 0
            op = None
        size = serialized_size(num_bits)
        if out is None:
            out = np.empty(size, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        _check(lib().lsmb_build_block(self.h, _p(data, u8p), op, key_len, n, num_bits, k, _p(out, u8p), out.size))
        return out

    def build_block_crc(self, data, num_bits, k, offsets=None, key_len=0, out=None):
        """build_block + the block's CRC-32 (lsmb_build_block_crc) -> (block, crc)."""
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n, op = offsets.size - 1, _p(offsets, u64p)
        else:
            n, op = (data.size // key_len if key_len else 0), None
        if out is None:
            out = np.empty(serialized_size(num_bits), dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        crc = ctypes.c_uint32()
        _check(lib().lsmb_build_block_crc(self.h, _p(data, u8p), op, key_len, n, num_bits, k, _p(out, u8p),
                                          out.size, ctypes.byref(crc)))
        return out, crc.value

    def crc32_dev(self, t, nbytes=None, crc=0, stream=None):
        """CRC-32 of a device tensor's bytes (lsmb_crc32_dev), appended to crc."""
        n = t.numel() * t.element_size() if nbytes is None else nbytes
        out = ctypes.c_uint32()
        _check(lib().lsmb_crc32_dev(self.h, crc, vp(t.data_ptr()), n, ctypes.byref(out), self._stream(stream)))
        return out.value

    def probe(self, filters, data, offsets=None, key_len=0):
        """filters: [(words uint64 array, num_bits, k)] -> uint8 [n, ceil(F/8)] mask."""
        F = len(filters)
        ws = [np.ascontiguousarray(f[0], dtype=np.uint64) for f in filters]
        arr = (u64p * F)(*[_p(w, u64p) for w in ws])
        nb = np.array([f[1] for f in filters], dtype=np.uint32)
        kk = np.array([f[2] for f in filters], dtype=np.uint32)
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n = offsets.size - 1
            op = _p(offsets, u64p)
        else:
            n = data.size // key_len if key_len else 0
            op = None
        out = np.zeros((n, (F + 7) // 8), dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        _check(lib().lsmb_probe(self.h, arr, _p(nb, u32p), _p(kk, u32p), F, _p(data, u8p), op, key_len, n,
                                _p(out, u8p)))
        return out

    # device-resident entry points (torch tensors) ------------------------------
    @staticmethod
    def _stream(stream):
        if stream is None:
            import torch
            return vp(torch.cuda.current_stream().cuda_stream)
        return vp(stream)

    def build_fixed_dev(self, keys, key_len, n, num_bits, k, words, stream=None):
        _check(lib().lsmb_build_fixed_dev(self.h, vp(keys.data_ptr()), key_len, n, num_bits, k,
                                          vp(words.data_ptr()), self._stream(stream)))

    def build_fixed_dev_sweep(self, keys, key_len, n, num_bits, k, words, sweep, stream=None):
        """One sweep of a partitioned build (lsmb_build_fixed_dev_sweep)."""
        _check(lib().lsmb_build_fixed_dev_sweep(self.h, vp(keys.data_ptr()), key_len, n, num_bits, k,
                                                vp(words.data_ptr()), int(sweep), self._stream(stream)))

    def build_var_dev(self, data, offsets, n, num_bits, k, words, stream=None):
        _check(lib().lsmb_build_var_dev(self.h, vp(data.data_ptr()), vp(offsets.data_ptr()), n, num_bits, k,
                                        vp(words.data_ptr()), self._stream(stream)))

    # BloomFilterBuilder::{new, add_key, build} (src/bloom/builder.rs:14-28):
    # `words` is output-only, every word of the filter (of the sweep's range)
    # is written; no zeroing pass, no read of the old words.
    def build_fixed_dev_new(self, keys, key_len, n, num_bits, k, words, stream=None):
        _check(lib().lsmb_build_fixed_dev_new(self.h, vp(keys.data_ptr() if n else 0), key_len, n, num_bits, k,
                                              vp(words.data_ptr()), self._stream(stream)))

    def build_fixed_dev_sweep_new(self, keys, key_len, n, num_bits, k, words, sweep, stream=None):
        _check(lib().lsmb_build_fixed_dev_sweep_new(self.h, vp(keys.data_ptr() if n else 0), key_len, n, num_bits,
                                                    k, vp(words.data_ptr()), int(sweep), self._stream(stream)))

    def build_var_dev_new(self, data, offsets, n, num_bits, k, words, stream=None):
        _check(lib().lsmb_build_var_dev_new(self.h, vp(data.data_ptr()), vp(offsets.data_ptr() if n else 0), n,
                                            num_bits, k, vp(words.data_ptr()), self._stream(stream)))

    def probe_dev(self, filters, data, n, out, offsets=None, key_len=0, stream=None):
        """filters: [(words tensor on device, num_bits, k)]."""
        F = len(filters)
        arr = (vp * F)(*[vp(f[0].data_ptr()) for f in filters])
        nb = np.array([f[1] for f in filters], dtype=np.uint32)
        kk = np.array([f[2] for f in filters], dtype=np.uint32)
        _check(lib().lsmb_probe_dev(self.h, arr, _p(nb, u32p), _p(kk, u32p), F, vp(data.data_ptr()),
                                    vp(offsets.data_ptr()) if offsets is not None else None, key_len, n,
                                    vp(out.data_ptr()), self._stream(stream)))

    def or_reduce_dev(self, dst, src, nwords, nsrc, stride_words, stream=None):
        _check(lib().lsmb_or_reduce_dev(self.h, vp(dst.data_ptr()), vp(src.data_ptr()), nwords, nsrc,
                                        stride_words, self._stream(stream)))

    def or_gather_dev(self, dst_ptr, src_ptrs, nwords, stream=None, status_ptr=0):
        """dst[i] = OR of src_j[i] over the raw device pointers src_ptrs (own or
        IPC-mapped peer memory), nwords u64 words (lsmb_or_gather_dev); with a
        merge's status words (status_ptr) a poisoned merge writes all-ones."""
        arr = (vp * len(src_ptrs))(*[vp(int(p)) for p in src_ptrs])
        _check(lib().lsmb_or_gather_dev(self.h, vp(int(dst_ptr)), arr, len(src_ptrs), int(nwords),
                                        vp(int(status_ptr or 0)), self._stream(stream)))

    def copy_slices_dev(self, dst_ptr, src_ptrs, slice_words, nwords, stream=None, status_ptr=0):
        """dst slice r = src_ptrs[r]'s slice r (u64 words) for every r whose source is
        not None/0: the merge's all-gather in one kernel (lsmb_copy_slices_dev)."""
        arr = (vp * len(src_ptrs))(*[vp(int(p or 0)) for p in src_ptrs])
        _check(lib().lsmb_copy_slices_dev(self.h, vp(int(dst_ptr)), arr, len(src_ptrs), int(slice_words), int(nwords),
                                          vp(int(status_ptr or 0)), vp(stream or 0)))

    def poison_fill_dev(self, words_ptr, nwords, status_ptr, stream=None):
        """The merge's last step: all-ones over nwords words if the merge is
        poisoned (lsmb_poison_fill_dev)."""
        _check(lib().lsmb_poison_fill_dev(self.h, vp(int(words_ptr)), int(nwords), vp(int(status_ptr)),
                                          vp(stream or 0)))

    def flag_signal_dev(self, flag_ptr, value, stream=None):
        """After the stream's prior work: *flag = value, system-scope release (lsmb_flag_signal_dev)."""
        _check(lib().lsmb_flag_signal_dev(self.h, vp(int(flag_ptr)), int(value) & 0xFFFFFFFF, vp(stream or 0)))

    def flag_wait_dev(self, flag_ptrs, value, status_ptr, timeout_ms=20000, poison_ptrs=None, stream=None):
        """Later work on the stream waits until every flag >= value; a timeout or
        a set poison word ends the wait and poisons the merge's status words
        (lsmb_flag_wait_dev)."""
        arr = (vp * len(flag_ptrs))(*[vp(int(p)) for p in flag_ptrs])
        parr = (vp * len(flag_ptrs))(*[vp(int(p)) for p in poison_ptrs]) if poison_ptrs else None
        if poison_ptrs and len(poison_ptrs) != len(flag_ptrs):
            raise ValueError("one poison word per flag")
        _check(lib().lsmb_flag_wait_dev(self.h, arr, parr, len(flag_ptrs), int(value) & 0xFFFFFFFF, int(timeout_ms),
                                        vp(int(status_ptr)), vp(stream or 0)))

    def merge_status(self, status_ptr, stream=None):
        """(poisoned, timed-out waits) of a merge's status words, after the
        stream's pending work (lsmb_merge_status: synchronises the stream)."""
        out = (ctypes.c_uint32 * 2)()
        _check(lib().lsmb_merge_status(self.h, vp(int(status_ptr)), vp(stream or 0), out))
        return int(out[0]), int(out[1])

    def ipc_import(self, handle):
        """Maps another process's device allocation (lsmb_ipc_import) -> base pointer (int)."""
        h = np.frombuffer(bytes(handle), dtype=np.uint8).copy()
        base = vp()
        _check(lib().lsmb_ipc_import(self.h, _p(h, u8p), ctypes.byref(base)))
        return int(base.value)

    def ipc_close(self, base):
        _check(lib().lsmb_ipc_close(self.h, vp(int(base))))

    def gen_key16_dev(self, seed, first, n, out, stream=None):
        _check(lib().lsmb_gen_key16_dev(self.h, seed, first, n, vp(out.data_ptr()), self._stream(stream)))

    def gen_splitmix_dev(self, seed, first, n, out, mod=0, add=0, stream=None):
        _check(lib().lsmb_gen_splitmix_dev(self.h, seed, first, n, mod, add, out.data_ptr(), self._stream(stream)))

    def gen_varlen_dev(self, n, first=0, device=None):
        """C4 keys [first, first+n) of tests/keygen.varlen on the device ->
        (data uint8 tensor, offsets int64 tensor [n+1], rebased to 0)."""
        import torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        lens = torch.empty(first + n, dtype=torch.int64, device=dev)
        self.gen_splitmix_dev(0x5EED0003, 0, first + n, lens, mod=249, add=8)
        offs = torch.zeros(first + n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=offs[1:])
        del lens
        o0, o1 = int(offs[first].item()), int(offs[first + n].item())
        w0, w1 = o0 // 8, (o1 + 7) // 8
        words = torch.empty(max(w1 - w0, 1), dtype=torch.int64, device=dev)
        self.gen_splitmix_dev(0x5EED0004, w0, w1 - w0, words)
        data = words.view(torch.uint8)[o0 - 8 * w0: o0 - 8 * w0 + (o1 - o0)]
        return data, (offs[first:] - o0).contiguous()

    def set_timing(self, on):
        """Per-build HIP events (lsmb_last_build_ms) on/off."""
        _check(lib().lsmb_set_timing(self.h, 1 if on else 0))

    def last_build_ms(self):
        a = (ctypes.c_float * 3)()
        _check(lib().lsmb_last_build_ms(self.h, a))
        return tuple(a)


class KeyStream:
    """Streaming ingestion (lsmb_stream): the flush's add_key loop
    (src/db/mod.rs:379-383 -> SSTableBuilder::add -> BloomFilterBuilder::add_key)
    with full staging chunks uploaded and built while keys keep arriving.
    finish_block() == BloomFilter::new(..) + inserts, serialized."""

    def __init__(self, ctx, num_bits, k):
        """ctx None: host-only (runs of at most host_max_keys() keys)."""
        h = vp()
        _check(lib().lsmb_stream_open(ctx.h if ctx else None, num_bits, k, ctypes.byref(h)))
        self.h, self.ctx, self.num_bits, self.k = h, ctx, num_bits, k

    def close(self):
        if self.h:
            lib().lsmb_stream_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, num_bits, k):
        _check(lib().lsmb_stream_reset(self.h, num_bits, k))
        self.num_bits, self.k = num_bits, k

    def add(self, key):
        a, n = _key(key)
        _check(lib().lsmb_stream_add(self.h, _p(a, u8p), n))

    def add_batch(self, data, offsets):
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        _check(lib().lsmb_stream_add_batch(self.h, _p(data, u8p), _p(offsets, u64p), offsets.size - 1))

    def count(self):
        return int(lib().lsmb_stream_count(self.h))

    def finish_block(self, out=None):
        if out is None:
            out = np.empty(serialized_size(self.num_bits), dtype=np.uint8)
        _check(lib().lsmb_stream_finish_block(self.h, _p(out, u8p), out.size))
        return out

    def finish_words(self):
        w = np.zeros(max(num_words(self.num_bits), 1), dtype=np.uint64)
        _check(lib().lsmb_stream_finish_words(self.h, _p(w, u64p)))
        return w[: num_words(self.num_bits)]


class FilterSet:
    """Device-resident SSTable filters with key ranges (lsmb_fset): the batched
    form of SSTable::get's range + bloom pre-check (src/sstable/reader.rs:192-199).

    probe(keys)[i] bit s = (min_s <= key_i <= max_s) and may_contain(filter s, key_i).
    """

    def __init__(self, ctx=None):
        self.ctx = ctx or default_context()
        h = vp()
        _check(lib().lsmb_fset_open(self.ctx.h, ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().lsmb_fset_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, block, min_key, max_key):
        """block: serialized filter bytes (BloomFilter::serialize) -> slot."""
        b, n = _key(block)
        lo, nlo = _key(min_key)
        hi, nhi = _key(max_key)
        return _check(lib().lsmb_fset_add(self.h, _p(b, u8p), n, _p(lo, u8p), nlo, _p(hi, u8p), nhi))

    def add_checked(self, block, crc, min_key, max_key):
        """add() that checks the block's CRC-32 on the device copy (lsmb_fset_add_crc)."""
        b, n = _key(block)
        lo, nlo = _key(min_key)
        hi, nhi = _key(max_key)
        return _check(lib().lsmb_fset_add_crc(self.h, _p(b, u8p), n, crc, _p(lo, u8p), nlo, _p(hi, u8p), nhi))

    def add_filter(self, filt, min_key, max_key):
        """filt: BloomFilter -> slot."""
        w = np.ascontiguousarray(filt.bits, dtype=np.uint64)
        if w.size == 0:
            w = np.zeros(1, np.uint64)
        lo, nlo = _key(min_key)
        hi, nhi = _key(max_key)
        return _check(lib().lsmb_fset_add_words(self.h, _p(w, u64p), filt.num_bits(), filt.num_hashes(),
                                                _p(lo, u8p), nlo, _p(hi, u8p), nhi))

    def remove(self, slot):
        _check(lib().lsmb_fset_remove(self.h, int(slot)))

    def live_mask(self):
        return int(lib().lsmb_fset_live_mask(self.h))

    def probe(self, data, offsets=None, key_len=0):
        """Packed host keys (as Context.probe) -> uint64 mask per key."""
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n = offsets.size - 1
            op = _p(offsets, u64p)
        else:
            n = data.size // key_len if key_len else 0
            op = None
        out = np.zeros(n, dtype=np.uint64)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        _check(lib().lsmb_fset_probe(self.h, _p(data, u8p), op, key_len, n, _p(out if n else np.zeros(1, np.uint64),
                                                                                u64p)))
        return out

    def probe_keys(self, keys):
        """list of bytes -> uint64 mask per key."""
        lens = np.array([len(k) for k in keys], dtype=np.uint64)
        offs = np.zeros(len(keys) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        return self.probe(np.frombuffer(b"".join(bytes(k) for k in keys), dtype=np.uint8), offs)

    def probe_dev(self, data, n, out, offsets=None, key_len=0, stream=None, row_bytes=8):
        """Device keys -> device answer rows: u64 per key (lsmb_fset_probe_dev),
        or row_bytes = 1 / 2 / 4 per key when every live slot fits them
        (lsmb_fset_probe_dev_rows)."""
        offs = vp(offsets.data_ptr()) if offsets is not None else None
        if row_bytes == 8:
            _check(lib().lsmb_fset_probe_dev(self.h, vp(data.data_ptr()), offs, key_len, n, vp(out.data_ptr()),
                                             Context._stream(stream)))
        else:
            _check(lib().lsmb_fset_probe_dev_rows(self.h, vp(data.data_ptr()), offs, key_len, n, vp(out.data_ptr()),
                                                  int(row_bytes), Context._stream(stream)))


def build_strategy(num_bits, n, k=7):
    """Device build strategy for (num_bits, k, n): lds / tiled / partition / atomic."""
    return lib().lsmb_build_strategy(num_bits, k, n).decode()


def crc32(data, crc=0):
    """CRC-32 of host bytes (lsmb_crc32; == zlib.crc32 == crc32fast::hash)."""
    a, n = _key(data)
    return int(lib().lsmb_crc32(crc, _p(a, u8p), n))


def crc32_combine(crc_a, crc_b, len_b):
    return int(lib().lsmb_crc32_combine(crc_a, crc_b, len_b))


def build_sweeps(num_bits, n, k=7):
    """Sweeps of the device build of n keys (1 unless partitioned in several)."""
    return int(lib().lsmb_build_sweeps(num_bits, k, n))


def sweep_words(num_bits, n, sweep, k=7):
    """[word_lo, word_hi): the filter words whose bits sweep `sweep` completes."""
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().lsmb_sweep_words(num_bits, k, n, int(sweep), ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def host_max_keys():
    """Host-memory builds of at most this many keys run the library's host loop."""
    return int(lib().lsmb_host_max_keys())


def set_host_max_keys(n):
    lib().lsmb_set_host_max_keys(int(n))


class Multi:
    """One process, several GPUs (lsmb_multi): a sharded build merged by an
    OR reduce-scatter over xGMI peer loads.  `devices` may repeat."""

    def __init__(self, devices):
        devices = list(devices)
        h = vp()
        arr = (ctypes.c_int * len(devices))(*devices)
        _check(lib().lsmb_multi_open(ctypes.byref(h), arr, len(devices)))
        self.h = h
        self.devices = devices

    def close(self):
        if self.h:
            lib().lsmb_multi_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self):
        return int(lib().lsmb_multi_size(self.h))

    def build_fixed_dev(self, keys, key_len, num_bits, k, words):
        """keys / words: per-shard torch tensors on the shards' devices; every
        words[g] ends holding the merged filter."""
        G = len(keys)
        karr = (vp * G)(*[vp(t.data_ptr()) for t in keys])
        warr = (vp * G)(*[vp(t.data_ptr()) for t in words])
        n = np.array([t.numel() // key_len if key_len else t.shape[0] for t in keys], dtype=np.uint64)
        _check(lib().lsmb_multi_build_fixed_dev(self.h, karr, _p(n, u64p), key_len, num_bits, k, warr))

    def build_block(self, data, num_bits, k, offsets=None, key_len=0, out=None):
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n, op = offsets.size - 1, _p(offsets, u64p)
        else:
            n, op = (data.size // key_len if key_len else 0), None
        if out is None:
            out = np.empty(serialized_size(num_bits), dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        _check(lib().lsmb_multi_build_block(self.h, _p(data, u8p), op, key_len, n, num_bits, k, _p(out, u8p),
                                            out.size))
        return out

    def last_ms(self):
        a = (ctypes.c_float * 3)()
        _check(lib().lsmb_multi_last_ms(self.h, a))
        return tuple(a)


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(-1)
    return _default_ctx


# ------------------------------------------------------------------ reference surface
class BloomFilter:
    """Mirror of `pub struct BloomFilter` (src/bloom/mod.rs:23-27): words + num_hashes + num_bits."""

    __slots__ = ("bits", "_k", "_nb")

    def __init__(self, bits, num_hashes, num_bits):
        self.bits = bits
        self._k = num_hashes
        self._nb = num_bits

    @classmethod
    def new(cls, expected_items, false_positive_rate):
        nb, k = params(expected_items, false_positive_rate)
        return cls(np.zeros(num_words(nb), dtype=np.uint64), k, nb)

    def insert(self, key):
        a, n = _key(key)
        _check(lib().lsmb_insert(_p(self.bits, u64p), self._nb, self._k, _p(a, u8p), n))

    def may_contain(self, key):
        a, n = _key(key)
        return bool(_check(lib().lsmb_may_contain(_p(self.bits, u64p), self._nb, self._k, _p(a, u8p), n)))

    def serialize(self):
        size = int(lib().lsmb_serialized_size(self._nb))
        out = np.zeros(size, dtype=np.uint8)
        _check(lib().lsmb_serialize(_p(self.bits, u64p), self._nb, self._k, _p(out, u8p), size))
        return out.tobytes()

    @classmethod
    def deserialize(cls, data):
        a, n = _key(data)
        k, nb, nw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().lsmb_deserialize_header(_p(a, u8p), n, ctypes.byref(k), ctypes.byref(nb), ctypes.byref(nw)))
        words = np.zeros(nw.value, dtype=np.uint64)
        _check(lib().lsmb_deserialize(_p(a, u8p), n, _p(words, u64p), nw.value))
        return cls(words, k.value, nb.value)

    def num_hashes(self):
        return self._k

    def num_bits(self):
        return self._nb

    # additive batched API (the reference has no multi-get)
    @staticmethod
    def may_contain_batch(filters, keys, ctx=None):
        """keys: list of bytes.  Returns uint8 [len(keys), ceil(F/8)] mask (GPU)."""
        ctx = ctx or default_context()
        offs = np.zeros(len(keys) + 1, dtype=np.uint64)
        if keys:
            offs[1:] = np.cumsum([len(k) for k in keys])
        data = np.frombuffer(b"".join(bytes(k) for k in keys), dtype=np.uint8)
        return ctx.probe([(f.bits, f._nb, f._k) for f in filters], data, offs)


class BloomFilterBuilder:
    """Mirror of `BloomFilterBuilder` (src/bloom/builder.rs:8-28).

    The reference inserts on the fly (builder.rs:21-23); this one buffers the
    run's keys in a packed arena and builds the whole filter in one GPU batch
    at `build()`.  The bits are identical.
    """

    def __init__(self, filt, ctx=None):
        self._filter = filt
        self._data = bytearray()
        self._offs = [0]
        self._ctx = ctx

    @classmethod
    def new(cls, estimated_keys, false_positive_rate, ctx=None):
        return cls(BloomFilter.new(estimated_keys, false_positive_rate), ctx)

    def add_key(self, key):
        self._data += bytes(key)
        self._offs.append(len(self._data))

    def _ctx_for(self, n):
        """The device context a build of n keys needs: None at or below the
        library's host threshold (SST-sized flushes stay on the host, no GPU
        required), else the GPU context (raises without a gfx950 device)."""
        if n <= host_max_keys():
            return None
        return self._ctx or default_context()

    def build(self):
        f = self._filter
        n = len(self._offs) - 1
        if n:
            ctx = self._ctx_for(n)
            offs = np.array(self._offs, dtype=np.uint64)
            data = np.frombuffer(bytes(self._data) or b"\0", dtype=np.uint8)
            _check(lib().lsmb_build_var(ctx.h if ctx else None, _p(data, u8p), _p(offs, u64p), n, f._nb, f._k,
                                        _p(f.bits, u64p)))
        return f

    def build_serialized(self):
        """build().serialize() in one call (lsmb_build_block): the bloom block
        SSTableBuilder::finish writes (src/sstable/builder.rs:177-179)."""
        f = self._filter
        n = len(self._offs) - 1
        ctx = self._ctx_for(n)
        offs = np.array(self._offs, dtype=np.uint64)
        data = np.frombuffer(bytes(self._data) or b"\0", dtype=np.uint8)
        out = np.empty(serialized_size(f._nb), dtype=np.uint8)
        _check(lib().lsmb_build_block(ctx.h if ctx else None, _p(data, u8p), _p(offs, u64p), 0, n, f._nb, f._k,
                                      _p(out, u8p), out.size))
        return out.tobytes()
