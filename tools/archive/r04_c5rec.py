#!/usr/bin/env python3
"""C5 shard (125 M 16-B keys into new(1e9, 0.01) = 2^32-1 bits) built two ways
for a rocprofv3 kernel trace: the fixed-16 path (each sweep's k_bin hashes
every key) and the same keys as var-len keys (k_hash_var writes 12-B walk
records once; each sweep's k_bin replays them).  The k_bin<Recs> time per
sweep prices the idea of emitting records in sweep 0 and replaying them in
sweep 1.  Checks that both filters are equal."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))

import bench  # noqa: E402


def main():
    import torch

    import lsmbloom
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 125_000_000
    nb, k = lsmbloom.params(1_000_000_000, 0.01)
    ctx = lsmbloom.Context(0)
    ctx.set_timing(False)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(bench.SEED_MEMBERS, 0, n, keys)
    offs = torch.arange(0, 16 * (n + 1), 16, dtype=torch.int64, device=dev)
    wa = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    wb = torch.empty_like(wa)
    flat = keys.view(-1)
    for _ in range(5):
        ctx.build_fixed_dev_new(keys, 16, n, nb, k, wa)
    for _ in range(5):
        ctx.build_var_dev_new(flat, offs, n, nb, k, wb)
    ctx.sync()
    torch.cuda.synchronize()
    print("num_bits", nb, "k", k, "filters equal:", bool(torch.equal(wa, wb)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
