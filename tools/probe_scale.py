#!/usr/bin/env python3
"""The C3 probe's fixed cost per launch vs its cost per key: lsmb_probe_dev
(k_probe_sliced) timed at several batch sizes Q against the same 8 SST
filters (bench.ProbeLegs), steady clocks (20 ms warm-up, >= 10 ms timed).
A line fit t(Q) = t0 + Q * c gives the launch-bound intercept t0 and the
per-key slope c.  Usage: tools/probe_scale.py [Q ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch

    import bench
    import lsmbloom
    qs = [int(float(x)) for x in sys.argv[1:]] or [1_000_000, 2_500_000, 5_000_000, 10_000_000, 20_000_000]
    dev = torch.device("cuda:0")
    ctx = lsmbloom.Context(0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    rows = []
    for q in qs:
        P = bench.ProbeLegs(ctx, dev, q, 8)
        ms = bench.timed_ms(P.probe, 5, 20, warm_ms=20, min_timed_ms=10)
        fms = bench.timed_ms(P.fset, 5, 20, warm_ms=20, min_timed_ms=10)
        rows.append({"Q": q, "probe_ms": round(ms, 5), "fset_ms": round(fms, 5)})
        print(json.dumps(rows[-1]), flush=True)
        P.close()
        del P
        torch.cuda.empty_cache()
    x = np.array([r["Q"] for r in rows], dtype=float)
    for key in ("probe_ms", "fset_ms"):
        y = np.array([r[key] for r in rows])
        c, t0 = np.polyfit(x, y, 1)
        print(json.dumps({"fit": key, "intercept_us": round(t0 * 1e3, 2), "ns_per_key": round(c * 1e6, 4),
                          "at_10M_ms": round(t0 + c * 1e7, 5)}))
    ctx.close()


if __name__ == "__main__":
    main()
