import os, sys, time, json
sys.path.insert(0, 'storage-engine_amd')
import torch, numpy as np, lsmbloom
ctx = lsmbloom.Context(0)
dev = torch.device('cuda:0')
for n in (150_000, 1_000_000, 3_500_000):
    nb, k = lsmbloom.params(n, 0.01)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
    w = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    res = {}
    for mode in ("default", "no_prehash", "atomic"):
        os.environ.pop("LSMB_FORCE_STRATEGY", None)
        os.environ.pop("LSMB_TILED_NO_PREHASH", None)
        if mode == "atomic": os.environ["LSMB_FORCE_STRATEGY"] = "atomic"
        if mode == "no_prehash": os.environ["LSMB_TILED_NO_PREHASH"] = "1"
        ts = []
        for r in range(12):
            w.zero_(); ctx.build_fixed_dev(keys, 16, n, nb, k, w); ctx.sync(); torch.cuda.synchronize()
            ts.append(ctx.last_build_ms()[0])
        res[mode] = round(float(np.median(ts[2:])), 4)
    print(json.dumps({"n": n, "num_bits": nb, "strategy": lsmbloom.build_strategy(nb, n), "kernel_ms": res}), flush=True)
