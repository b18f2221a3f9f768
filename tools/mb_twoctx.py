"""Microbenchmark: do back-to-back C2 builds gain from running two at once?

Pass A (k_bin) is bound by LDS instruction issue, pass B (k_apply) by HBM;
each takes a whole CU's LDS per workgroup, so a CU runs one of them at a
time, but the chip could run one build's pass B beside the next build's
pass A.  Two contexts (each its own workspace) on two streams build C2
(100 M 16-B keys into new(1e8, 0.01)) alternately; every result is compared
with a sequential build.  Prints one JSON line per configuration.
Usage: python tools/mb_twoctx.py [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "storage-engine_amd"))
import lsmbloom  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--lags", type=int, nargs="*", default=[50_000, 100_000, 200_000, 400_000, 800_000])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = args.n
    nb, k = lsmbloom.params(n, 0.01)
    nw = lsmbloom.num_words(nb)
    ctxs = [lsmbloom.Context(0) for _ in range(2)]
    keys = [torch.empty((n, 16), dtype=torch.uint8, device=dev) for _ in range(2)]
    for i, kk in enumerate(keys):
        ctxs[0].gen_key16_dev(0x5EED0001 + i, 0, n, kk)
    words = [torch.empty(nw, dtype=torch.int64, device=dev) for _ in range(2)]
    ref = [torch.empty(nw, dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    for i in range(2):
        ctxs[0].build_fixed_dev_new(keys[i], 16, n, nb, k, ref[i])
    ctxs[0].sync()
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]

    def run(mode, reps, lag=0):
        torch.cuda.synchronize()
        t = time.perf_counter()
        builds = 0
        if lag:  # stream 1 starts `lag` clock cycles after stream 0 (phase offset)
            with torch.cuda.stream(streams[1]):
                torch.cuda._sleep(lag)
        for r in range(reps):
            if mode == "one":
                ctxs[0].build_fixed_dev_new(keys[r & 1], 16, n, nb, k, words[r & 1], stream=streams[0].cuda_stream)
                builds += 1
            else:
                for i in range(2):
                    ctxs[i].build_fixed_dev_new(keys[i], 16, n, nb, k, words[i], stream=streams[i].cuda_stream)
                builds += 2
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3 / builds, builds

    t = time.perf_counter()
    torch.cuda._sleep(1_000_000)
    torch.cuda.synchronize()
    print(json.dumps({"sleep_1e6_cycles_ms": round((time.perf_counter() - t) * 1e3, 3)}), flush=True)
    for mode, lag in [("one", 0), ("two", 0)] + [("two", x) for x in args.lags] + [("one", 0)]:
        run(mode, 3, lag)
        ms, b = run(mode, args.reps, lag)
        exact = all(torch.equal(words[i], ref[i]) for i in range(2))
        print(json.dumps({"mode": mode, "lag_cycles": lag, "builds": b, "ms_per_build": round(ms, 4),
                          "Mkeys_s": round(n / ms / 1e3, 1), "words_exact": exact}), flush=True)
        if not exact:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
