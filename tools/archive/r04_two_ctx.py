#!/usr/bin/env python3
"""C2 builds from two contexts at once (two flush threads, each with its own
lsmb_ctx, workspace and stream, as the Rust shim's thread-local contexts would
run them): does pass B of one build overlap pass A of the other?  Times K
builds serial on one context against K builds alternating between two
contexts on two streams, and checks both filters against the C2 fixture."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))

import bench  # noqa: E402


def main():
    import torch

    import lsmbloom
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 100_000_000
    nb, k = lsmbloom.params(n, 0.01)
    ctxs = [lsmbloom.Context(0), lsmbloom.Context(0)]
    for c in ctxs:
        c.set_timing(False)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctxs[0].gen_key16_dev(bench.SEED_MEMBERS, 0, n, keys)
    words = [torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()

    def build(i):
        ctxs[i].build_fixed_dev_new(keys, 16, n, nb, k, words[i], stream=streams[i].cuda_stream)

    K = 40
    for _ in range(20):
        build(0)
        build(1)
    torch.cuda.synchronize()
    for rep in range(2):
        t = time.perf_counter()
        for _ in range(K):
            build(0)
        torch.cuda.synchronize()
        serial = (time.perf_counter() - t) / K * 1e3
        t = time.perf_counter()
        for j in range(K):
            build(j & 1)
        torch.cuda.synchronize()
        two = (time.perf_counter() - t) / K * 1e3
        print("rep %d: one context %.4f ms/build, two contexts %.4f ms/build (%.1f%%)"
              % (rep, serial, two, 100 * (two / serial - 1)), flush=True)
    ok = [bench.fixture_check(w, "c2", nb) for w in words]
    print("both filters equal the C2 fixture:", ok, flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
