"""Deterministic synthetic key sets (BASELINE.md generators), vectorised in numpy."""
import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
VAR_LEN_SEED = 0x5EED0003
VAR_DATA_SEED = 0x5EED0004


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + GOLD
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def key16(seed, first, n):
    """[n,16] uint8: LE64(sm(seed+2i)) || LE64(sm(seed+2i+1))."""
    i = np.arange(first, first + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        a = splitmix64(np.uint64(seed) + np.uint64(2) * i)
        b = splitmix64(np.uint64(seed) + np.uint64(2) * i + np.uint64(1))
    return np.stack([a, b], axis=1).astype("<u8").view(np.uint8).reshape(n, 16)


def stream_bytes(seed, nbytes):
    w = splitmix64(np.uint64(seed) + np.arange((nbytes + 7) // 8, dtype=np.uint64))
    return w.astype("<u8").view(np.uint8)[:nbytes].copy()


def varlen(n, first=0):
    """C4 keys: len_i = 8 + sm(0x5EED0003+i) % 249; packed data from the 0x5EED0004 stream.
    Returns (data uint8, offsets uint64[n+1]) for keys [first, first+n) of the global stream
    (data is the slice of the global packed stream, offsets rebased to 0)."""
    idx = np.arange(0, first + n, dtype=np.uint64)
    lens = np.uint64(8) + splitmix64(np.uint64(VAR_LEN_SEED) + idx) % np.uint64(249)
    offs = np.zeros(first + n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    o0, o1 = int(offs[first]), int(offs[first + n])
    w0 = o0 // 8
    words = splitmix64(np.uint64(VAR_DATA_SEED) + np.arange(w0, (o1 + 7) // 8, dtype=np.uint64))
    data = words.astype("<u8").view(np.uint8)[o0 - 8 * w0: o0 - 8 * w0 + (o1 - o0)].copy()
    return data, (offs[first:] - np.uint64(o0)).astype(np.uint64)


def ascii_keys(fmt, rng):
    """Reference-test style keys, e.g. ascii_keys('key_{}', range(100)) -> (data, offsets)."""
    ks = [fmt.format(i).encode() for i in rng]
    return pack(ks)


def pack(keys):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(k) for k in keys]) if keys else []
    data = np.frombuffer(b"".join(keys), dtype=np.uint8).copy()
    return data, offs
