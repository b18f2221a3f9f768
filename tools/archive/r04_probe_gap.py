#!/usr/bin/env python3
"""Where the C3 probe's per-call time goes beyond its kernel: the bench's
back-to-back lsmb_probe_dev calls (HIP events around 200 calls), the host's
enqueue rate for the same calls, tiny batches (the per-call floor), and the
same calls replayed from a captured hipGraph."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402


def main():
    import torch

    import lsmbloom
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = lsmbloom.Context(0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    ctx.set_timing(False)
    P = bench.ProbeLegs(ctx, dev, 10_000_000, 8)
    N = 200
    ms = bench.timed_ms(P.probe, 10, N)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        P.probe()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("probe 10M x 8: %.4f ms/call (events); host enqueue %.4f ms/call; wall %.4f ms/call"
          % (ms, (t1 - t0) * 1e3 / N, (t2 - t0) * 1e3 / N), flush=True)
    small = bench.ProbeLegs(ctx, dev, 4096, 8)
    print("probe 4096 x 8: %.4f ms/call (events)" % bench.timed_ms(small.probe, 10, N), flush=True)
    # the same calls captured once and replayed (no per-call host launch work)
    g = torch.cuda.CUDAGraph()
    P.probe()
    torch.cuda.synchronize()
    reps = 20
    with torch.cuda.graph(g):
        for _ in range(reps):
            P.probe()
    g.replay()
    torch.cuda.synchronize()
    gms = bench.timed_ms(g.replay, 3, 10) / reps
    print("probe 10M x 8 from a graph: %.4f ms/call" % gms, flush=True)
    ok = bench._sha(P.out) == bench.c3_fixture()["probe_mask_sha256"] if bench.c3_fixture() else None
    print("answers equal the fixture after the replays:", ok, flush=True)
    P.close()
    small.close()
    ctx.close()


if __name__ == "__main__":
    main()
