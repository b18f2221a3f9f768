"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ODIR = os.path.join(ROOT, "oracle")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    subprocess.run(["make", "-s", "-C", ODIR], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(ODIR, "liboracle.so")
    if not os.path.exists(path):
        build()
    _lib = _bind(path)
    return _lib


NATIVE_FLAGS = ["-O3", "-march=native", "-fPIC", "-std=c11", "-D_GNU_SOURCE"]


def load_native(outdir=None):
    """The oracle compiled on THIS host with -O3 -march=native (BASELINE.md's
    CPU-baseline flags): bench.py's cpu_baseline leg builds it on the GPU box,
    whose CPU differs from the build container's.  Returns (Oracle, how);
    falls back to the portable liboracle.so when no C compiler is present."""
    import shutil
    import tempfile
    cc = shutil.which(os.environ.get("CC", "gcc")) or shutil.which("cc")
    if cc:
        d = outdir or tempfile.mkdtemp(prefix="lsmb_oracle_")
        out = os.path.join(d, "liboracle_native.so")
        r = subprocess.run([cc] + NATIVE_FLAGS + ["-shared", "-o", out, os.path.join(ODIR, "bloom_oracle.c"),
                                                  "-lm", "-lpthread"], capture_output=True, text=True)
        if r.returncode == 0:
            return _bind(out), "oracle/bloom_oracle.c, %s %s (built on this host)" % (os.path.basename(cc),
                                                                                        " ".join(NATIVE_FLAGS[:2]))
    return load(), "oracle/liboracle.so (portable -O3; no C compiler for a -march=native build)"


def _bind(path):
    lib = ctypes.CDLL(path)
    V, I, Z, D = None, ctypes.c_int, ctypes.c_size_t, ctypes.c_double
    U32, U64 = ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "oracle_xxh3_128": (V, [u8p, Z, u64p, u64p]),
        "oracle_bloom_params": (I, [U64, D, u32p, u32p]),
        "oracle_bloom_positions": (V, [u8p, Z, U32, U32, u32p]),
        "oracle_bloom_insert": (V, [u64p, U32, U32, u8p, Z]),
        "oracle_bloom_may_contain": (I, [u64p, U32, U32, u8p, Z]),
        "oracle_bloom_build_fixed": (V, [u8p, U32, U64, U32, U32, u64p]),
        "oracle_bloom_build_var": (V, [u8p, u64p, U64, U32, U32, u64p]),
        "oracle_bloom_probe": (V, [ctypes.POINTER(u64p), u32p, u32p, U32, u8p, u64p, U32, U64, u8p]),
        "oracle_bloom_serialize": (U64, [u64p, U32, U32, u8p]),
        "oracle_bloom_deserialize": (I, [u8p, U64, u32p, u32p, u32p, u64p]),
        "oracle_gen_key16": (V, [U64, U64, U64, u8p]),
        "oracle_bloom_build_fixed_mt": (I, [u8p, U32, U64, U32, U32, u64p, I]),
        "oracle_bloom_build_var_mt": (I, [u8p, u64p, U64, U32, U32, u64p, I]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return Oracle(lib)


def _p(a, t):
    return a.ctypes.data_as(t)


def _buf(b):
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)  # +1 so empty keys have a pointer
    return a


class Oracle:
    def __init__(self, lib):
        self.lib = lib

    def xxh3_128(self, b):
        a = _buf(b)
        lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.oracle_xxh3_128(_p(a, u8p), len(b), ctypes.byref(lo), ctypes.byref(hi))
        return lo.value, hi.value

    def params(self, n, fpr):
        nb, k = ctypes.c_uint32(), ctypes.c_uint32()
        rc = self.lib.oracle_bloom_params(n, fpr, ctypes.byref(nb), ctypes.byref(k))
        if rc != 0:
            raise ValueError("BloomFilter::new panics for n=%r fpr=%r" % (n, fpr))
        return nb.value, k.value

    def positions(self, key, num_bits, k):
        a = _buf(key)
        out = np.zeros(k, dtype=np.uint32)
        self.lib.oracle_bloom_positions(_p(a, u8p), len(key), num_bits, k, _p(out, u32p))
        return [int(x) for x in out]

    @staticmethod
    def nwords(num_bits):
        return (num_bits + 63) // 64

    def build_fixed(self, keys, key_len, num_bits, k, words=None):
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = keys.size // key_len if key_len else 0
        if words is None:
            words = np.zeros(self.nwords(num_bits), dtype=np.uint64)
        self.lib.oracle_bloom_build_fixed(_p(keys, u8p), key_len, n, num_bits, k, _p(words, u64p))
        return words

    def build_fixed_mt(self, keys, key_len, num_bits, k, threads, words=None):
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = keys.size // key_len if key_len else 0
        if words is None:
            words = np.zeros(self.nwords(num_bits), dtype=np.uint64)
        rc = self.lib.oracle_bloom_build_fixed_mt(_p(keys, u8p), key_len, n, num_bits, k,
                                                  _p(words, u64p), threads)
        assert rc == 0
        return words

    def build_var(self, data, offsets, num_bits, k, words=None):
        data = np.ascontiguousarray(np.frombuffer(bytes(data) + b"\0", np.uint8)
                                    if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if words is None:
            words = np.zeros(self.nwords(num_bits), dtype=np.uint64)
        self.lib.oracle_bloom_build_var(_p(data, u8p), _p(offsets, u64p), offsets.size - 1,
                                        num_bits, k, _p(words, u64p))
        return words

    def build_var_mt(self, data, offsets, num_bits, k, threads, words=None):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if words is None:
            words = np.zeros(self.nwords(num_bits), dtype=np.uint64)
        rc = self.lib.oracle_bloom_build_var_mt(_p(data, u8p), _p(offsets, u64p), offsets.size - 1,
                                                num_bits, k, _p(words, u64p), threads)
        assert rc == 0
        return words

    def insert(self, words, num_bits, k, key):
        a = _buf(key)
        self.lib.oracle_bloom_insert(_p(words, u64p), num_bits, k, _p(a, u8p), len(key))

    def may_contain(self, words, num_bits, k, key):
        a = _buf(key)
        return bool(self.lib.oracle_bloom_may_contain(_p(words, u64p), num_bits, k, _p(a, u8p), len(key)))

    def probe(self, filters, data, offsets=None, key_len=0, n=None):
        """filters: list of (words, num_bits, k). Returns uint8 [n, ceil(F/8)] mask."""
        F = len(filters)
        arr = (u64p * F)(*[_p(w, u64p) for (w, _, _) in filters])
        nb = np.array([f[1] for f in filters], dtype=np.uint32)
        kk = np.array([f[2] for f in filters], dtype=np.uint32)
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n = offsets.size - 1
            op = _p(offsets, u64p)
        else:
            n = data.size // key_len if n is None else n
            op = None
        stride = (F + 7) // 8
        out = np.zeros((n, stride), dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        self.lib.oracle_bloom_probe(arr, _p(nb, u32p), _p(kk, u32p), F, _p(data, u8p), op,
                                    key_len, n, _p(out, u8p))
        return out

    def serialize(self, words, num_bits, k):
        nw = self.nwords(num_bits)
        out = np.zeros(12 + 8 * nw, dtype=np.uint8)
        m = self.lib.oracle_bloom_serialize(_p(words, u64p), num_bits, k, _p(out, u8p))
        assert m == out.size
        return out.tobytes()

    def deserialize(self, data):
        """Returns (k, num_bits, words) or raises ValueError(code)."""
        a = _buf(data)
        k, nb, nw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        rc = self.lib.oracle_bloom_deserialize(_p(a, u8p), len(data), ctypes.byref(k),
                                               ctypes.byref(nb), ctypes.byref(nw), None)
        if rc != 0:
            raise ValueError(rc)
        words = np.zeros(nw.value, dtype=np.uint64)
        self.lib.oracle_bloom_deserialize(_p(a, u8p), len(data), ctypes.byref(k), ctypes.byref(nb),
                                          ctypes.byref(nw), _p(words, u64p))
        return k.value, nb.value, words

    def key16(self, seed, first, n):
        out = np.zeros((n, 16), dtype=np.uint8)
        self.lib.oracle_gen_key16(seed, first, n, _p(out, u8p))
        return out
