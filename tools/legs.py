#!/usr/bin/env python3
"""One bench leg in a process of its own, for per-leg rocprofv3 passes
(tools/profile_legs.sh): the leg's data is set up exactly as bench.py sets it
up, then the leg's device work runs --reps times.  Nothing else launches
kernels after the setup, so a pass's per-kernel means belong to this leg.

  c2        C2: 100 M 16-B keys into new(1e8, 0.01), lsmb_build_fixed_dev_new
  exact10   the C2 keys into num_bits = 1e9, k = 7
  c5        C5 shard: 125 M keys into new(1e9, 0.01) = 2^32-1 bits (2 sweeps)
  c5_full   C5 on one GPU: all 1e9 keys into the same filter, sweep by sweep
            (lsmb_build_fixed_dev_sweep_new, as each rank builds at N > 1)
  c4        C4: 100 M var-len keys (8-256 B) into new(1e8, 0.01), lsmb_build_var_dev_new
  probe     C3: 10 M keys x 8 new(1000, 0.01) filters, lsmb_probe_dev
  fset      the same through the device filter set (range pre-check + bloom)
  fset_mixed  a filter set of two sizes (4 x new(1000) + 4 x new(4000))
  fset_rows1  the fset leg with one-byte answer rows (lsmb_fset_probe_dev_rows)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402  (the legs' shared setup: ProbeLegs, seeds)

LEGS = ("c2", "exact10", "c5", "c5_full", "c4", "probe", "fset", "fset_mixed", "fset_rows1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("leg", choices=LEGS)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    import lsmbloom
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = lsmbloom.Context(0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    ctx.set_timing(False)
    leg = args.leg
    if leg in ("c2", "exact10", "c5"):
        n = 125_000_000 if leg == "c5" else 100_000_000
        if leg == "exact10":
            nb, k = 10 * n, 7
        else:
            nb, k = lsmbloom.params(10**9 if leg == "c5" else n, 0.01)
        keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
        ctx.gen_key16_dev(bench.SEED_MEMBERS, 0, n, keys)
        words = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)

        def run():
            ctx.build_fixed_dev_new(keys, 16, n, nb, k, words)
    elif leg == "c5_full":
        n = 1_000_000_000
        nb, k = lsmbloom.params(n, 0.01)
        keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
        ctx.gen_key16_dev(bench.SEED_MEMBERS, 0, n, keys)
        words = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
        nsw = lsmbloom.build_sweeps(nb, n, k)

        def run():
            for s in range(nsw):
                ctx.build_fixed_dev_sweep_new(keys, 16, n, nb, k, words, s)
    elif leg == "c4":
        n = 100_000_000
        data, offs = ctx.gen_varlen_dev(n, device=dev)
        nb, k = lsmbloom.params(n, 0.01)
        words = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)

        def run():
            ctx.build_var_dev_new(data, offs, n, nb, k, words)
    else:
        P = bench.ProbeLegs(ctx, dev, 10_000_000, 8)
        run = getattr(P, leg)
    torch.cuda.synchronize()
    for _ in range(args.reps):
        run()
    torch.cuda.synchronize()
    ctx.sync()
    print("leg %s: %d reps done" % (leg, args.reps), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
