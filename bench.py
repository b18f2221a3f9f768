#!/usr/bin/env python3
"""bench.py — BASELINE metric: Bloom build (+ batched probe), Mkeys/s, device-resident.

A step = one device-resident build of a fresh filter over this rank's batch of
synthetic 16-byte keys (BASELINE configs[1] = C2 at N=1: 100 M keys into
BloomFilter::new(1e8, 0.01) -> 956 715 292 bits, k = 7), i.e. zero the words,
hash every key, set its 7 bits — and, for N > 1 GPUs, the bitwise-OR allreduce
that merges the ranks' partial filters (RCCL has no BOR op: all_to_all
reduce-scatter + native OR kernel + all_gather).  Weak scaling: each rank owns
--keys-per-gpu keys of one global run; the filter is sized for the global run
(for N >= 5 that saturates at 2^32-1 bits, the C5 filter, src/bloom/mod.rs:49).

Also reported (extra keys on the same JSON line):
  probe        C3: 10 M 16-B lookup keys x 8 SSTable filters (new(1000, 0.01)), Mkeys/s
  roofline     the build kernels vs 8 TB/s HBM, algorithmic bytes per build
  cpu_baseline the CPU oracle (C restatement of src/bloom, "port") on a bounded sample
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "storage-engine_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
SEED_MEMBERS = 0x5EED0001
SEED_FRESH = 0x5EED0002


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--keys-per-gpu", type=int, default=100_000_000)
    ap.add_argument("--probe-keys", type=int, default=10_000_000)
    ap.add_argument("--probe-filters", type=int, default=8)
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time box")
    ap.add_argument("--verify", action="store_true", help="check the built filter against the oracle")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end measurement")
    ap.add_argument("--no-varlen", action="store_true", help="skip the C4 variable-length build leg")
    ap.add_argument("--varlen-keys", type=int, default=100_000_000)
    ap.add_argument("--filter-keys", type=int, default=0, help="size the filter for this many keys (default: all ranks' keys)")
    return ap.parse_args()


def cpu_baseline(num_bits, k, budget_s):
    """Oracle (C restatement of src/bloom, single thread) building the C2-size
    filter from the first S keys of the same workload, S grown until ~budget_s."""
    import numpy as np
    import oracle_ct
    orc = oracle_ct.load()
    words = np.zeros((num_bits + 63) // 64, dtype=np.uint64)
    done, t_used, chunk = 0, 0.0, 1_000_000
    keys = None
    while t_used < budget_s and done < 100_000_000:
        keys = orc.key16(SEED_MEMBERS, done, chunk)
        t0 = time.perf_counter()
        orc.build_fixed(keys, 16, num_bits, k, words=words)
        t_used += time.perf_counter() - t0
        done += chunk
    st = {"value": round(done / t_used / 1e6, 3), "unit": "Mkeys/s", "cores": 1, "kind": "port",
          "sample": "first %d keys of the C2 workload into the full C2 filter (%d bits, k=%d), "
                    "1 thread, oracle/bloom_oracle.c -O3" % (done, num_bits, k)}
    # all-cores variant (the box's CPU share: at most 16 threads)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    words[:] = 0
    n_mt = min(done * threads, 20_000_000)
    keys = orc.key16(SEED_MEMBERS, 0, n_mt)
    t0 = time.perf_counter()
    orc.build_fixed_mt(keys, 16, num_bits, k, threads, words=words)
    dt = time.perf_counter() - t0
    st["multi_thread"] = {"value": round(n_mt / dt / 1e6, 3), "cores": threads,
                          "sample": "first %d keys, atomic fetch_or" % n_mt}
    return st


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import lsmbloom

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctx = lsmbloom.Context(local)
    stream = torch.cuda.current_stream(dev)

    npg = args.keys_per_gpu
    total = npg * world
    # --filter-keys: size the filter for a larger global run than this job's
    # keys (rehearses the per-GPU build of an N-GPU run on one GPU; C5's
    # 1e9-key filter saturates at 2^32-1 bits).  Reported in config.
    nb, k = lsmbloom.params(args.filter_keys or total, 0.01)
    nw = lsmbloom.num_words(nb)
    keys = torch.empty((npg, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(SEED_MEMBERS, rank * npg, npg, keys)
    words = torch.zeros(nw, dtype=torch.int64, device=dev)
    from lsmbloom import dist as ldist

    def step():
        words.zero_()
        ctx.build_fixed_dev(keys, 16, npg, nb, k, words)
        if world > 1:
            ldist.or_allreduce_(words, ctx=ctx)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    ctx.set_timing(False)  # no timing markers between the kernels of a timed step
    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    value = total * args.steps / dt / 1e6

    # per-kernel times (HIP events on the build stream), averaged over `steps` builds
    ctx.set_timing(True)
    kt = np.zeros(3)
    for _ in range(args.steps):
        words.zero_()
        ctx.build_fixed_dev(keys, 16, npg, nb, k, words)
        ctx.sync()
        torch.cuda.synchronize(dev)
        kt += np.array(ctx.last_build_ms())
    kt /= args.steps
    strategy = lsmbloom.build_strategy(nb, npg)
    alg_bytes = 16 * npg + 8 * nw
    achieved = alg_bytes / (kt[0] * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "build (%s: k_bin + k_apply)" % strategy,
            "algorithmic_bytes": alg_bytes, "kernel_ms": round(float(kt[0]), 4),
            "pass_a_ms": round(float(kt[1]), 4), "pass_b_ms": round(float(kt[2]), 4)}

    out = {"metric": "bloom build + batched probe, Mkeys/s device-resident, at 1/2/4/8 MI355X",
           "value": round(value, 2), "unit": "Mkeys/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8/u64 (XXH3-128 + bit OR)",
           "data": "synthetic key16(0x5EED0001, i) = splitmix64 stream, generated on device",
           "config": {"workload": "C2 (configs[1]): build BloomFilter::new(%d, 0.01) from %d 16-B keys per GPU"
                                  % (total, npg),
                      "keys_per_gpu": npg, "global_keys": total, "num_bits": nb, "k": k,
                      "filter_bytes": 8 * nw, "strategy": strategy, "parallelism": "dp%d" % world}}
    if args.filter_keys:
        out["config"]["filter_sized_for_keys"] = args.filter_keys
    out["roofline"] = roof

    if world > 1:
        # Multi-GPU self-check (outside the timed region): one more sharded
        # step (build + OR-allreduce); rank 0 then rebuilds the whole global
        # key set alone, 100 M keys at a time, and compares every word.  OR is
        # associative and idempotent, so the merged filter must be identical.
        step()
        torch.cuda.synchronize(dev)
        if rank == 0:
            try:
                ref = torch.zeros_like(words)
                for first in range(0, total, npg):
                    m = min(npg, total - first)
                    ctx.gen_key16_dev(SEED_MEMBERS, first, m, keys[:m])
                    ctx.build_fixed_dev(keys[:m], 16, m, nb, k, ref)
                ctx.sync()
                torch.cuda.synchronize(dev)
                out["multi_gpu_merged_equals_single_gpu_build"] = bool(torch.equal(ref, words))
                del ref
                ctx.gen_key16_dev(SEED_MEMBERS, rank * npg, npg, keys)  # this rank's shard again
            except Exception as e:  # report, never lose the bench line
                out["multi_gpu_check_error"] = repr(e)[:200]
        dist.barrier()

    if args.verify and rank == 0 and world == 1:
        import oracle_ct
        orc = oracle_ct.load()
        host = orc.key16(SEED_MEMBERS, 0, npg)
        ref = orc.build_fixed_mt(host, 16, nb, k, 16)
        out["verified_bit_exact"] = bool(np.array_equal(words.cpu().numpy().view(np.uint64), ref))

    if not args.no_probe:
        out["probe"] = bench_probe(ctx, dev, args)
    if not args.no_e2e and rank == 0 and world == 1:
        out["e2e"] = bench_e2e(ctx, keys, npg, nb, k)

    del keys
    words = None
    torch.cuda.empty_cache()
    if not args.no_varlen and world == 1:
        out["varlen"] = bench_varlen(ctx, dev, args)
    tr = committed_traffic()
    if tr:
        out["roofline"]["traffic"] = tr["bytes"]
        out["roofline"]["traffic_source"] = tr["source"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(nb, k, args.cpu_seconds)
        out["cpu_baseline"]["gpu_over_cpu_1thread"] = round(value / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def bench_e2e(ctx, keys, n, nb, k, reps=3):
    """Keys in host memory -> serialized bloom block in host memory: the flush
    path (SSTableBuilder::finish, src/sstable/builder.rs:177-182).  One
    lsmb_build_block call: chunked H2D of the keys overlapped with the build
    kernels, then D2H of the words straight into the block (no serialize copy).
    Measured with pageable key memory (a memtable arena) and pinned key memory."""
    import numpy as np
    import torch

    import lsmbloom
    size = lsmbloom.serialized_size(nb)
    res = {"what": "host keys -> H2D (chunked, overlapped) -> build -> D2H into the serialized block "
                   "(lsmb_build_block)", "h2d_bytes": n * 16, "d2h_bytes": size - 12, "serialized_bytes": size}
    host = keys.cpu().numpy().reshape(-1)
    for name, src in (("pageable", host), ("pinned", None)):
        if src is None:
            pin = torch.empty(host.size, dtype=torch.uint8).pin_memory()
            pin.numpy()[:] = host
            src = pin.numpy()
        block = np.empty(size, dtype=np.uint8)
        block[:] = 0  # fault the pages in before timing
        ctx.build_block(src, nb, k, key_len=16, out=block)  # warm-up (staging allocations)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ctx.build_block(src, nb, k, key_len=16, out=block)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        res[name] = {"ms": round(t * 1e3, 2), "value": round(n / t / 1e6, 1), "unit": "Mkeys/s",
                     "pcie_GBs": round((n * 16 + size) / t / 1e9, 1)}
    res["value"] = res["pageable"]["value"]
    res["unit"] = "Mkeys/s"
    # SST-sized flushes: one lsmb_build_block call per table, sized like
    # SSTableBuilder::with_estimated_keys (builder.rs:74); latency per call
    # (H2D, kernels, D2H, sync) next to the 1-thread CPU oracle on the same keys.
    import oracle_ct
    orc = oracle_ct.load()
    small = []
    for m in (1000, 100_000, 1_000_000):
        nb_m, k_m = lsmbloom.params(m, 0.01)
        ks = np.ascontiguousarray(host[: m * 16])
        blk = np.empty(lsmbloom.serialized_size(nb_m), dtype=np.uint8)
        ctx.build_block(ks, nb_m, k_m, key_len=16, out=blk)
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            ctx.build_block(ks, nb_m, k_m, key_len=16, out=blk)
            ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        ref = orc.build_fixed(ks.reshape(m, 16), 16, nb_m, k_m)
        tc = time.perf_counter() - t0
        small.append({"keys": m, "strategy": lsmbloom.build_strategy(nb_m, m),
                      "gpu_ms": round(float(np.median(ts)) * 1e3, 3), "cpu_oracle_1t_ms": round(tc * 1e3, 3),
                      "bit_exact": bool(np.array_equal(np.frombuffer(blk[12:].tobytes(), dtype=np.uint64), ref))})
    res["sst_flush_latency"] = small
    return res


def bench_varlen(ctx, dev, args):
    """C4 (configs[3]): 100 M variable-length keys (8-256 B, mean 132 B; the
    tests/keygen.varlen stream), packed data + offsets resident in HBM, into
    BloomFilter::new(1e8, 0.01)."""
    import numpy as np
    import torch

    import lsmbloom
    n = args.varlen_keys
    data, offs = ctx.gen_varlen_dev(n, device=dev)
    nb, k = lsmbloom.params(n, 0.01)
    nw = lsmbloom.num_words(nb)
    words = torch.zeros(nw, dtype=torch.int64, device=dev)

    def step():
        words.zero_()
        ctx.build_var_dev(data, offs, n, nb, k, words)

    ctx.set_timing(False)
    for _ in range(max(1, args.warmup // 2)):
        step()
    torch.cuda.synchronize(dev)
    steps = max(1, args.steps // 2)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    ctx.set_timing(True)
    kt = np.zeros(3)
    for _ in range(steps):
        words.zero_()
        ctx.build_var_dev(data, offs, n, nb, k, words)
        ctx.sync()
        kt += np.array(ctx.last_build_ms())
    kt /= steps
    ctx.set_timing(False)
    alg = int(data.numel()) + 8 * (n + 1) + 8 * nw
    res = {"workload": "C4 (configs[3]): %d var-len keys (8-256 B, %.1f B mean) into new(%d, 0.01) (%d bits, k=%d)"
                       % (n, data.numel() / n, n, nb, k),
           "value": round(n / dt / 1e6, 1), "unit": "Mkeys/s", "ms_per_step": round(dt * 1e3, 3),
           "kernel_ms": round(float(kt[0]), 4), "pass_a_ms": round(float(kt[1]), 4),
           "pass_b_ms": round(float(kt[2]), 4), "algorithmic_bytes": alg,
           "achieved_GBs": round(alg / (kt[0] * 1e-3) / 1e9, 1),
           "frac": round(alg / (kt[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "strategy": lsmbloom.build_strategy(nb, n)}
    del data, offs, words
    torch.cuda.empty_cache()
    return res


def committed_traffic():
    """HBM bytes per C2 build from the committed rocprofv3 PMC summary
    (profiles/traffic.json, written by tools/prof_summary.py --json from separate
    FETCH_SIZE / WRITE_SIZE passes of this bench; FETCH_SIZE doubled per the
    gfx950 note in MI355X_MICROARCH.md).  None if absent."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    t = json.load(open(p))
    return {"bytes": t.get("build_bytes"), "source": "%s (%s)" % (os.path.relpath(p, ROOT), t.get("profile"))}


def bench_probe(ctx, dev, args):
    """C3: Q lookup keys (50% members drawn across the F filters, 50% fresh)
    against F per-SSTable filters sized like SSTableBuilder::new (1000 keys, 0.01)."""
    import numpy as np
    import torch

    import lsmbloom
    F, Q = args.probe_filters, args.probe_keys
    nb, k = lsmbloom.params(1000, 0.01)
    nw = lsmbloom.num_words(nb)
    filt = []
    members = torch.empty((F * 1000, 16), dtype=torch.uint8, device=dev)
    for f in range(F):
        ctx.gen_key16_dev(0xF000 + f, 0, 1000, members[f * 1000:(f + 1) * 1000])
        w = torch.zeros(nw, dtype=torch.int64, device=dev)
        ctx.build_fixed_dev(members[f * 1000:(f + 1) * 1000], 16, 1000, nb, k, w)
        filt.append((w, nb, k))
    q = torch.empty((Q, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(SEED_FRESH, 0, Q, q)
    g = torch.Generator(device="cpu").manual_seed(1)
    sel = torch.randint(0, F * 1000, (Q // 2,), generator=g).to(dev)
    q[: Q // 2] = members[sel]
    out = torch.zeros((Q, (F + 7) // 8), dtype=torch.uint8, device=dev)
    for _ in range(max(1, args.warmup)):
        ctx.probe_dev(filt, q, Q, out, key_len=16)
    torch.cuda.synchronize(dev)
    st = torch.cuda.Event(enable_timing=True)
    en = torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(args.steps):
        ctx.probe_dev(filt, q, Q, out, key_len=16)
    en.record()
    torch.cuda.synchronize(dev)
    ms = st.elapsed_time(en) / args.steps
    alg = Q * 16 + Q * out.shape[1] + F * (12 + 8 * nw)
    hits = int((out[: Q // 2] != 0).all(dim=1).sum().item())
    res = {"workload": "C3 (configs[2]): %d 16-B keys x %d filters new(1000, 0.01) (%d bits, k=%d)"
                       % (Q, F, nb, k),
           "value": round(Q / (ms * 1e-3) / 1e6, 2), "unit": "Mkeys/s", "ms": round(ms, 4),
           "achieved_GBs": round(alg / (ms * 1e-3) / 1e9, 1), "member_rows_all_hit": hits == Q // 2}
    # The same batch through the device-resident filter set (lsmb_fset): per
    # key and SSTable, min_key <= key <= max_key && may_contain — the checks
    # SSTable::get makes (src/sstable/reader.rs:192-199) — for all 8 tables.
    fs = lsmbloom.FilterSet(ctx)
    slots = []
    for f in range(F):
        rows = members[f * 1000:(f + 1) * 1000].cpu().numpy()
        srt = sorted(bytes(r) for r in rows)
        slots.append(fs.add_filter(lsmbloom.BloomFilter(filt[f][0].cpu().numpy().view(np.uint64), k, nb),
                                   srt[0], srt[-1]))
    fout = torch.zeros(Q, dtype=torch.int64, device=dev)
    for _ in range(max(1, args.warmup)):
        fs.probe_dev(q, Q, fout, key_len=16)
    torch.cuda.synchronize(dev)
    st.record()
    for _ in range(args.steps):
        fs.probe_dev(q, Q, fout, key_len=16)
    en.record()
    torch.cuda.synchronize(dev)
    fms = st.elapsed_time(en) / args.steps
    # a member row's own table must answer 1 (range and bloom); here sel // 1000
    own = (fout[: Q // 2] >> torch.tensor(slots, device=dev)[sel // 1000]) & 1
    res["fset"] = {"what": "lsmb_fset_probe_dev: range pre-check + bloom, %d tables, u64 mask per key" % F,
                   "value": round(Q / (fms * 1e-3) / 1e6, 2), "unit": "Mkeys/s", "ms": round(fms, 4),
                   "member_rows_own_table_hit": bool(own.all().item())}
    fs.close()
    return res


if __name__ == "__main__":
    main()
