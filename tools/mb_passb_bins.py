"""Measurement: pass B (k_apply) time against the bin count, at a fixed 700 M
positions (100 M 16-B keys, k = 7) and filter sizes of 640..1024 2^20-bit bins.
Pass B runs one workgroup per bin (all of a CU's LDS), so if its time is set
by rounds of 256 workgroups, C2's 912 bins (3.56 rounds) pay a tail round at
56 % occupancy; if it is set by the bytes, the time is flat.  One JSON line
per size.  Usage: python tools/mb_passb_bins.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "storage-engine_amd"))
import lsmbloom  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bins", type=int, nargs="*",
                    default=[640, 700, 767, 768, 769, 800, 850, 896, 912, 960, 1000, 1023])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, k = 100_000_000, 7
    ctx = lsmbloom.Context(0)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    for b in args.bins:
        nb = b * (1 << 20) - 4096
        words = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
        ctx.build_fixed_dev_new(keys, 16, n, nb, k, words)
        ctx.sync()
        ctx.set_timing(True)
        kt = np.zeros(3)
        for _ in range(args.reps):
            ctx.build_fixed_dev_new(keys, 16, n, nb, k, words)
            ctx.sync()
            kt += np.array(ctx.last_build_ms())
        ctx.set_timing(False)
        kt /= args.reps
        print(json.dumps({"bins": b, "num_bits": nb, "sweeps": lsmbloom.build_sweeps(nb, n, k),
                          "strategy": lsmbloom.build_strategy(nb, n, k), "kernel_ms": round(kt[0], 4),
                          "pass_a_ms": round(kt[1], 4), "pass_b_ms": round(kt[2], 4),
                          "pass_b_us_per_bin_round": round(kt[2] * 1e3 / -(-b // 256), 2)}), flush=True)
        del words
    return 0


if __name__ == "__main__":
    sys.exit(main())
