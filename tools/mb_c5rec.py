"""Microbenchmark: the C5 shard (125 M 16-B keys into 2^32-1 bits, two sweeps)
built from the keys (each sweep's pass A hashes every key again) and from
12-B walk records (the keys hashed once by k_hash_var, both sweeps' pass A
replaying the records) — the var-len entry point over the same keys laid out
as 16-B var-len keys.  Both must give the same words.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel split.
Usage: python tools/mb_c5rec.py [--reps 10]
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--n", type=int, default=125_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, nb, k = args.n, 4294967295, 7
    nw = lsmbloom.num_words(nb)
    ctx = lsmbloom.Context(0)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    offs = torch.arange(0, 16 * (n + 1), 16, dtype=torch.int64, device=dev)
    w_key = torch.empty(nw, dtype=torch.int64, device=dev)
    w_rec = torch.empty(nw, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    runs = {"keys": lambda: ctx.build_fixed_dev_new(keys, 16, n, nb, k, w_key),
            "records": lambda: ctx.build_var_dev_new(keys.view(-1), offs, n, nb, k, w_rec)}
    for name, fn in list(runs.items()) * 2:
        fn()
        ctx.sync()
        torch.cuda.synchronize()
        ctx.set_timing(True)
        t = time.perf_counter()
        tot = [0.0, 0.0, 0.0]
        for _ in range(args.reps):
            fn()
            ctx.sync()
            tot = [a + b for a, b in zip(tot, ctx.last_build_ms())]
        torch.cuda.synchronize()
        ctx.set_timing(False)
        print(json.dumps({"form": name, "kernel_ms": round(tot[0] / args.reps, 4),
                          "pass_a_ms": round(tot[1] / args.reps, 4), "pass_b_ms": round(tot[2] / args.reps, 4),
                          "wall_ms": round((time.perf_counter() - t) * 1e3 / args.reps, 4)}), flush=True)
    same = torch.equal(w_key, w_rec)
    print(json.dumps({"words_equal": same}), flush=True)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
