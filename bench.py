#!/usr/bin/env python3
"""bench.py — BASELINE metric: Bloom build (+ batched probe), Mkeys/s, device-resident.

A step = one device-resident build of a fresh filter over this rank's shard of
synthetic 16-byte keys, i.e. zero the words, hash every key, set its 7 bits —
and, for N > 1 GPUs, the bitwise-OR allreduce that merges the ranks' partial
filters (RCCL has no BOR op: all_to_all reduce-scatter + native OR kernel +
all_gather).
  N = 1: C2 (BASELINE configs[1]): 100 M keys into BloomFilter::new(1e8, 0.01)
         -> 956 715 292 bits, k = 7.
  N > 1: C5 (configs[4]): 1e9 keys split over the N ranks (strong scaling) into
         new(1e9, 0.01) = 2^32-1 bits (the saturated u32, src/bloom/mod.rs:49).
`--gpus N` launched without torchrun starts the N rank processes itself.

Also reported (extra keys on the same JSON line):
  probe        C3: 10 M 16-B lookup keys x 8 SSTable filters (new(1000, 0.01)), Mkeys/s
  roofline     the build kernels vs 8 TB/s HBM, algorithmic bytes per build
  cpu_baseline the CPU oracle (C restatement of src/bloom, "port") on a bounded sample,
               and C1 (configs[0]) build + probe, 1 thread and all cores
  c2_exact_10_bits_per_key  the C2 keys into num_bits = 10 n, k = 7
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
    ap.add_argument("--warmup", type=int, default=20)  # ~28 ms of C2 steps: the clock has ramped (tools/archive/r04_warm.sh)
    ap.add_argument("--global-keys", type=int, default=0,
                    help="keys of the whole run, split over the ranks (default: 1e8 = C2 at N=1, 1e9 = C5 at N>1)")
    ap.add_argument("--keys-per-gpu", type=int, default=0,
                    help="weak scaling instead: this many keys per rank (overrides --global-keys)")
    ap.add_argument("--backend", default="auto",
                    help="N>1 merge: auto (RCCL and IPC both set up; the untimed calibration checks that they agree "
                         "word for word and times the faster), nccl (RCCL collectives only), gloo (host-staged), "
                         "ipc (peer loads over IPC-mapped device words, device-ordered phases), auto-gloo (auto "
                         "with gloo in RCCL's place).  nccl and auto need one GPU per rank")
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="let auto run with more ranks than visible GPUs (as ipc: a one-GPU rehearsal; the line then "
                         "says ranks_per_gpu > 1 and is not a scaling figure)")
    ap.add_argument("--inject-merge-fault", action="store_true", help=argparse.SUPPRESS)  # tests: a wrong merge
    ap.add_argument("--inject-ipc-poison", action="store_true", help=argparse.SUPPRESS)  # tests: IPC merge poisoned
    ap.add_argument("--probe-keys", type=int, default=10_000_000)
    ap.add_argument("--probe-filters", type=int, default=8)
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--accumulate", action="store_true",
                    help="time zero + the OR-accumulate build (lsmb_build_fixed_dev) instead of the fresh build")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time box")
    ap.add_argument("--verify", action="store_true", help="check the built filter against the oracle")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end measurement")
    ap.add_argument("--no-varlen", action="store_true", help="skip the C4 variable-length build leg")
    ap.add_argument("--no-exact10", action="store_true", help="skip the C2 exact 10 bits/key leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 shard leg (N = 1)")
    ap.add_argument("--no-c5-full", action="store_true",
                    help="skip the C5 full leg (N = 1: all 1e9 C5 keys on one GPU, the N > 1 curve's 1-GPU point)")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1-on-the-GPU leg")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: build the whole filter, then OR-allreduce it (no per-sweep overlap)")
    ap.add_argument("--step-form", default="auto", choices=("auto", "overlapped", "pipelined", "serial"),
                    help="N > 1: the step form to time (auto: the fastest of the calibration)")
    ap.add_argument("--varlen-keys", type=int, default=100_000_000)
    ap.add_argument("--filter-keys", type=int, default=0, help="size the filter for this many keys (default: the global run)")
    ap.add_argument("--detail-out", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full record (every leg with its prose) is written; stdout gets the compact line")
    return ap.parse_args()


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: start N rank processes (one per
    GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their env) and wait for them.
    Nothing in this parent touches a GPU.  Rank 0 prints the JSON line; the
    exit code is the first failing rank's (the others are then stopped)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 1
                for q in alive:
                    q.terminate()
        time.sleep(0.1)
    return rc


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """The host CPUs this process may run on: sched_getaffinity, capped by a
    cgroup CPU quota if one is set; with the physical cores behind them
    (distinct (physical id, core id) of /proc/cpuinfo) and the CPU model."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    cores, cur = set(), {}
    try:
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (x.strip() for x in line.split(":", 1))
                cur[k] = v
            elif cur:
                if int(cur.get("processor", -1)) in aff:
                    cores.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur and int(cur.get("processor", -1)) in aff:
            cores.add((cur.get("physical id"), cur.get("core id")))
    except (OSError, ValueError):
        pass
    use = min(len(aff), quota) if quota else len(aff)
    return {"threads": max(1, use), "affinity_cpus": len(aff), "cgroup_cpu_quota": quota,
            "physical_cores": len(cores) or None, "cpu": cpu_model()}


def cpu_baseline(num_bits, k, budget_s):
    """Oracle (C restatement of src/bloom, built on this host with -O3
    -march=native: BASELINE.md) on the box's host cores, reported beside the
    GPU numbers: the C2-size filter built from the first S keys of the same
    workload (S grown until ~budget_s, 1 thread; then every host CPU this
    process may use, with atomic fetch_or), and C1 (configs[0]): build + probe
    of 100 k 16-B keys, 1 thread and all of those CPUs."""
    import numpy as np
    import oracle_ct
    orc, how = oracle_ct.load_native()
    hc = host_cpus()
    words = np.zeros((num_bits + 63) // 64, dtype=np.uint64)
    done, t_used, chunk = 0, 0.0, 1_000_000
    keys = None
    while t_used < budget_s and done < 100_000_000:
        keys = orc.key16(SEED_MEMBERS, done, chunk)
        t0 = time.perf_counter()
        orc.build_fixed(keys, 16, num_bits, k, words=words)
        t_used += time.perf_counter() - t0
        done += chunk
    threads = hc["threads"]
    st = {"value": round(done / t_used / 1e6, 3), "unit": "Mkeys/s", "cores": 1, "kind": "port",
          "cpu": hc["cpu"], "host": hc, "oracle_build": how,
          "sample": "first %d keys of the C2 workload into the full C2 filter (%d bits, k=%d), "
                    "1 thread, %s" % (done, num_bits, k, how)}
    words[:] = 0
    n_mt = min(max(done * threads // 4, 4_000_000), 100_000_000)
    keys = orc.key16(SEED_MEMBERS, 0, n_mt)
    orc.build_fixed_mt(keys[:1_000_000], 16, num_bits, k, threads, words=words)  # warm-up: threads, pages
    words[:] = 0
    t0 = time.perf_counter()
    orc.build_fixed_mt(keys, 16, num_bits, k, threads, words=words)
    dt = time.perf_counter() - t0
    st["multi_thread"] = {"value": round(n_mt / dt / 1e6, 3), "cores": threads,
                          "sample": "first %d keys, atomic fetch_or, %d threads = every CPU this process may use "
                                    "(affinity %d, cgroup quota %s; %s physical cores)"
                                    % (n_mt, threads, hc["affinity_cpus"], hc["cgroup_cpu_quota"],
                                       hc["physical_cores"])}
    st["c1"] = cpu_c1(orc, threads)
    return st


def cpu_c1(orc, threads, reps=20):
    """C1 (BASELINE configs[0]): BloomFilter::new(100000, 0.01) built from 100 k
    key16 members, then 100 k members + 100 k non-members probed; the oracle
    on 1 thread and on `threads` threads (probe: key chunks per thread, the
    ctypes calls release the GIL)."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    n = 100_000
    nb, k = orc.params(n, 0.01)
    mem = orc.key16(SEED_MEMBERS, 0, n)
    non = orc.key16(SEED_FRESH, 0, n)
    q = np.concatenate([mem, non])
    t0 = time.perf_counter()
    for _ in range(reps):
        ref = orc.build_fixed(mem, 16, nb, k)
    tb1 = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        ans = orc.probe([(ref, nb, k)], q, key_len=16)
    tp1 = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        orc.build_fixed_mt(mem, 16, nb, k, threads)
    tbm = (time.perf_counter() - t0) / reps
    parts = np.array_split(q, threads)
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        for _ in range(reps):
            list(ex.map(lambda p: orc.probe([(ref, nb, k)], p, key_len=16), parts))
        tpm = (time.perf_counter() - t0) / reps
    fp = int(ans[n:, 0].sum())
    return {"workload": "C1 (configs[0]): build new(100000, 0.01) (%d bits, k=%d) from 100000 key16 members; "
                        "probe 100000 members + 100000 non-members" % (nb, k),
            "build_1t": {"ms": round(tb1 * 1e3, 3), "value": round(n / tb1 / 1e6, 2), "unit": "Mkeys/s"},
            "probe_1t": {"ms": round(tp1 * 1e3, 3), "value": round(2 * n / tp1 / 1e6, 2), "unit": "Mkeys/s"},
            "build_mt": {"ms": round(tbm * 1e3, 3), "value": round(n / tbm / 1e6, 2), "unit": "Mkeys/s",
                         "cores": threads},
            "probe_mt": {"ms": round(tpm * 1e3, 3), "value": round(2 * n / tpm / 1e6, 2), "unit": "Mkeys/s",
                         "cores": threads},
            "members_all_hit": bool(ans[:n, 0].all()), "non_member_fp": fp}


def shard(total, world, rank):
    return total * rank // world, total * (rank + 1) // world


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    import numpy as np
    import torch
    import torch.distributed as dist

    import lsmbloom
    from lsmbloom import dist as ldist

    ndev = torch.cuda.device_count()
    backend = args.backend
    if world > 1 and backend in ("nccl", "auto") and world > ndev:
        if backend == "nccl" or not args.allow_shared_gpu:
            # a misconfigured HIP_VISIBLE_DEVICES must not produce an "N-GPU"
            # line measured on fewer GPUs
            print("bench.py: %d ranks need %d GPUs for --backend %s, %d visible (--allow-shared-gpu, --backend ipc "
                  "or auto-gloo run ranks sharing a GPU)" % (world, world, backend, ndev), file=sys.stderr)
            sys.exit(2)
        backend = "ipc"  # ranks sharing a GPU (one-GPU rehearsal): RCCL refuses them, IPC does not
    dev = torch.device("cuda", local % max(1, ndev))
    torch.cuda.set_device(dev)
    side_group = None  # gloo group of the IPC merge's handle exchange (auto: beside RCCL)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend in ("nccl", "auto"):
            dist.init_process_group("nccl", device_id=dev)
            if backend == "auto":
                side_group = dist.new_group(backend="gloo")
        elif backend == "auto-gloo":  # auto's two-merge path with gloo in RCCL's place (one-GPU tests)
            dist.init_process_group("gloo")
            side_group = dist.new_group(backend="gloo")
        else:  # gloo; ipc: gloo exchanges the handles, the words move by peer loads
            dist.init_process_group("gloo" if backend == "ipc" else backend)
    ctx = lsmbloom.Context(dev.index)
    # One explicit stream for all of this rank's work: on torch's default (the
    # legacy null) stream, the library maps stream NULL to its context's
    # blocking stream, so each step's words.zero_() and build would sit on
    # two streams with an implicit synchronisation between every launch
    # (C2 step 1.500 -> ~1.46 ms on one stream; tools/graph_ab.py).
    torch.cuda.set_stream(torch.cuda.Stream(dev))

    # Workload.  N = 1: C2 (configs[1]), 100 M keys into new(1e8, 0.01).
    # N > 1: C5 (configs[4]), 1e9 keys split over the ranks (strong scaling),
    # filter new(1e9, 0.01) = 2^32-1 bits.  --keys-per-gpu: weak scaling.
    if args.keys_per_gpu:
        total = args.keys_per_gpu * world
        lo, hi = rank * args.keys_per_gpu, (rank + 1) * args.keys_per_gpu
        scaling = "weak"
    else:
        total = args.global_keys or (100_000_000 if world == 1 else 1_000_000_000)
        lo, hi = shard(total, world, rank)
        scaling = "strong"
    npg = hi - lo
    nmax = max(shard(total, world, r)[1] - shard(total, world, r)[0] for r in range(world))
    nb, k = lsmbloom.params(args.filter_keys or total, 0.01)
    nw = lsmbloom.num_words(nb)
    cfg_name = {100_000_000: "C2 (configs[1])", 1_000_000_000: "C5 (configs[4])"}.get(total, "custom")
    keys = torch.empty((npg, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(SEED_MEMBERS, lo, npg, keys)
    words = torch.zeros(nw, dtype=torch.int64, device=dev)
    host_coll = world > 1 and backend not in ("nccl", "auto")

    # BloomFilterBuilder::{new, add_key, build} (src/bloom/builder.rs:14-28):
    # lsmb_build_fixed_dev_new writes every word of the filter (output-only
    # words: no zeroing pass, pass B never reads the old words).
    def build():
        if args.accumulate:  # measurement: the OR-accumulate entry point after a zeroing pass
            words.zero_()
            ctx.build_fixed_dev(keys, 16, npg, nb, k, words)
        else:
            ctx.build_fixed_dev_new(keys, 16, npg, nb, k, words)

    # The N > 1 merges, each fn(lo, hi, stream) = OR-allreduce of words[lo:hi]
    # after the stream's pending work:
    #   rccl  all_to_all reduce-scatter + native OR + all_gather (lsmbloom.dist)
    #   ipc   peer loads over IPC-mapped words, phases ordered by device flags
    #         (lsmbloom.dist.IpcMerge; no collective library on the data path)
    # --backend auto (default) sets up both; the untimed calibration checks that
    # they merge to the same words and times the faster one.
    merges, merge_notes, ipc = {}, {}, None
    if world > 1:
        if backend in ("nccl", "auto", "gloo", "auto-gloo"):
            def m_coll(a, b, stream):
                with torch.cuda.stream(stream):
                    ldist.or_allreduce_(words[a:b], ctx=ctx)
            merges["rccl" if backend in ("nccl", "auto") else "gloo"] = m_coll
        if backend in ("ipc", "auto", "auto-gloo"):
            err = None
            try:
                ipc = ldist.IpcMerge(words, ctx, group=side_group, ordered="device")
            except Exception as e:  # e.g. no IPC mapping between these GPUs: keep RCCL
                err = repr(e)[:200]
            ok = torch.tensor([0 if err else 1], dtype=torch.int32)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=side_group)
            if int(ok.item()) == 1:
                merges["ipc"] = lambda a, b, stream: ipc.allreduce(a, b, stream=stream)
            else:
                merge_notes["ipc_error"] = err or "failed on another rank"
                if ipc:
                    for base in ipc.bases:
                        ctx.ipc_close(base)
                    ipc = None
    form = next(iter(merges), None)

    # N > 1 step: the partitioned build runs in sweeps (C5: 2 x 256 MiB word
    # ranges); sweep s's range is final when its pass B ends, so its OR-allreduce
    # runs on a side stream while sweep s+1 builds (lsmb_build_fixed_dev_sweep).
    nsw = lsmbloom.build_sweeps(nb, npg, k)
    ranges = [lsmbloom.sweep_words(nb, npg, s, k) for s in range(nsw)]
    overlap = world > 1 and nsw > 1 and not args.no_overlap
    side = torch.cuda.Stream(dev) if overlap else None
    sweep_ev = [torch.cuda.Event() for _ in range(nsw)]
    merge_ev = [torch.cuda.Event() for _ in range(nsw)]
    pending = [False] * nsw  # pipelined steps: range s's last merge may still run on `side`
    # Step forms: "serial" (build, then merge the whole filter), "overlapped"
    # (range s merges on a side stream while sweep s+1 builds; the step ends
    # when every merge has), "pipelined" (the same, and the step does not wait
    # for its last range's merge: the next step's sweep 0, which rewrites only
    # range 0, runs under it, and sweep s waits only for range s's previous
    # merge — back-to-back flushes / compactions as a stream).  Every form's
    # work is inside the timed region, which ends with a device synchronise.
    mode = "overlapped" if overlap else "serial"

    def allreduce(f=None):
        if world > 1:
            merges[f or form](0, nw, torch.cuda.current_stream(dev))

    def step(md=None, f=None):
        f = f or form
        md = md or mode
        main = torch.cuda.current_stream(dev)
        if md == "serial":
            if side is not None and any(pending):  # a full rewrite waits for pipelined merges
                main.wait_stream(side)
                pending[:] = [False] * nsw
            build()
            allreduce(f)
            return
        for s, (a, b) in enumerate(ranges):
            if pending[s]:
                main.wait_event(merge_ev[s])  # range s's previous merge is done with these words
            ctx.build_fixed_dev_sweep_new(keys, 16, npg, nb, k, words, s)
            sweep_ev[s].record(main)
            side.wait_event(sweep_ev[s])
            merges[f](a, b, side)
            if md == "pipelined":
                merge_ev[s].record(side)
                pending[s] = True
        if md != "pipelined":
            main.wait_stream(side)
            pending[:] = [False] * nsw

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if host_coll else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    ctx.set_timing(False)  # no timing markers between the kernels of a timed step
    calib = None
    if ipc is not None:
        # A merge takes milliseconds: a phase wait this long means a peer never
        # signalled (or its flags are not visible here); the merge is then
        # dropped below instead of stalling every step.
        ipc.timeout_ms = 3000
        if args.inject_ipc_poison and rank == world - 1:
            # tests: this rank's merge status starts poisoned, as after a peer
            # timed out on it; every rank's IPC merge then ends all-ones
            ipc.flags[3] = 1
            torch.cuda.synchronize(dev)
    if world > 1 and len(merges) > 1:
        # The merges must agree word for word (one serial step each, untimed,
        # before any warm-up) and the IPC merge's waits must all have been
        # met; otherwise only RCCL is timed.
        snaps, failed = {}, None
        for f in merges:
            try:
                step("serial", f)
                torch.cuda.synchronize(dev)
            except Exception as e:  # an IPC merge error drops IPC (its waits time out on the peers)
                if f != "ipc":
                    raise
                failed = repr(e)[:200]
            barrier()
            snaps[f] = words.clone()
        names = list(snaps)
        agree = failed is None and all(torch.equal(snaps[names[0]], snaps[x]) for x in names[1:])
        del snaps
        if failed:
            merge_notes["ipc_error"] = failed
        elif ipc is not None and ipc.status()[0]:
            agree = False
            merge_notes["ipc_error"] = "merge poisoned in the agreement step (%d flag waits timed out)" % ipc.timeouts()
        t = torch.tensor([1 if agree else 0], dtype=torch.int32, device=dev if not host_coll else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        merge_notes["merges_agree"] = bool(t.item())
        if not merge_notes["merges_agree"]:
            merges.pop("ipc", None)
            form = next(iter(merges))
    modes = ("overlapped", "pipelined", "serial") if overlap else ("serial",)
    if args.step_form != "auto" and overlap:
        modes = (args.step_form,)
        mode = args.step_form
    forms = [(f, md) for f in (merges or [None]) for md in modes]
    for i in range(args.warmup):
        step(forms[i % len(forms)][1], forms[i % len(forms)][0])
    barrier()
    if len(forms) > 1:
        # Overlapped / pipelined vs serial and RCCL vs IPC: the overlapped
        # collective shares the CUs with pass A, whose workgroups each need a
        # whole CU's LDS, and the merges' speed depends on the node's links.
        # Time a few steps of each form (untimed for the metric; the max over
        # ranks, so every rank picks the same) and time the fastest.
        def timed(f, md, reps):
            barrier()
            t = time.perf_counter()
            for _ in range(reps):
                step(md, f)
            barrier()
            return max_over_ranks(time.perf_counter() - t) / reps * 1e3
        reps = max(2, min(5, args.steps))
        cal = {(f, md): timed(f, md, reps) for f, md in forms}
        form, mode = min(cal, key=cal.get)
        calib = {"%s_%s_ms_per_step" % (f, md): round(v, 4) for (f, md), v in cal.items()}
        calib.update({"steps_each": reps, "timed_form": mode, "timed_merge": form})
    if args.step_form != "auto" and overlap:
        calib = dict(calib or {}, timed_form=mode, timed_merge=form, step_form="forced by --step-form")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    ms = dt / args.steps * 1e3
    value = total * args.steps / dt / 1e6
    build_ms = coll_ms = serial_ms = 0.0
    if world > 1:
        # Split (outside the timed region): the same steps run serially —
        # build, then the full-filter OR-allreduce — timed by events.
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        barrier()
        t1 = time.perf_counter()
        for e0, e1, e2 in ev:
            e0.record()
            build()
            e1.record()
            allreduce()
            e2.record()
        barrier()
        serial_ms = max_over_ranks(time.perf_counter() - t1) / args.steps * 1e3
        build_ms = max_over_ranks(sum(a.elapsed_time(b) for a, b, _ in ev) / args.steps)
        coll_ms = max_over_ranks(sum(b.elapsed_time(c) for _, b, c in ev) / args.steps)

    # per-kernel times (HIP events on the build stream), averaged over `steps` builds
    ctx.set_timing(True)
    kt = np.zeros(3)
    for _ in range(args.steps):
        build()
        ctx.sync()
        torch.cuda.synchronize(dev)
        kt += np.array(ctx.last_build_ms())
    kt /= args.steps
    ctx.set_timing(False)
    strategy = lsmbloom.build_strategy(nb, npg, k)
    alg_bytes = 16 * npg + 8 * nw
    # C2 at N = 1; a C5 shard (125 M keys into 2^32-1 bits) at N = 8
    main_leg = {(100_000_000, 956715292): "c2", (125_000_000, 4294967295): "c5"}.get((npg, nb))
    roof = leg_roofline(main_leg, alg_bytes, kt[0], "build (%s: k_bin + k_apply + k_ovf_apply)" % strategy)
    roof.update({"algorithmic_bytes_per_key": round(alg_bytes / npg, 3), "pass_a_ms": round(float(kt[1]), 4),
                 "pass_b_ms": round(float(kt[2]), 4)})
    if world == 1 and npg == 100_000_000:
        roof["hash_walk_floor"] = dict(HASH_WALK_FLOOR, frac_of_hbm_roofline_at_that_time=round(
            alg_bytes / (HASH_WALK_FLOOR["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
        roof["hash_walk_floor"]["phase"] = PASS_A_PHASE

    out = {"metric": "bloom build + batched probe, Mkeys/s device-resident, at 1/2/4/8 MI355X",
           "value": round(value, 2), "unit": "Mkeys/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
           "scaling": scaling, "vs_baseline": None, "dtype": "u8/u64 (XXH3-128 + bit OR)",
           "data": "synthetic key16(0x5EED0001, i) = splitmix64 stream, generated on device",
           "config": {"workload": "%s: build BloomFilter::new(%d, 0.01) from %d 16-B keys, %d per GPU"
                                  % (cfg_name, args.filter_keys or total, total, nmax),
                      "keys_per_gpu": nmax, "global_keys": total, "num_bits": nb, "k": k,
                      "filter_bytes": 8 * nw, "strategy": strategy, "scaling": scaling,
                      "entry_point": "lsmb_build_fixed_dev_new (BloomFilter::new + insert per key; "
                                     "output-only words, every word written once)" if world == 1 else
                                     "lsmb_build_fixed_dev_sweep_new per sweep + OR-allreduce",
                      "parallelism": "dp%d" % world}}
    if args.filter_keys:
        out["config"]["filter_sized_for_keys"] = args.filter_keys
    out["roofline"] = roof
    if world > 1:
        moved = 2 * (world - 1) / world * 8 * nw
        out["config"]["backend"] = backend
        out["config"]["physical_gpus"] = min(world, ndev)
        out["config"]["ranks_per_gpu"] = -(-world // max(1, ndev))
        merge_what = {"ipc": "ipc: peer loads over IPC-mapped words (OR gather reduce-scatter + copy all-gather), "
                             "phases ordered by device flags",
                      "rccl": "rccl: all_to_all reduce-scatter + native OR kernel + all_gather",
                      "gloo": "gloo: host-staged collectives + native OR kernel"}
        out["step_split"] = {"build_ms": round(build_ms, 4), "or_allreduce_ms": round(coll_ms, 4),
                             "what": "serial steps (untimed pass), slowest rank: device build (fresh) / "
                                     "bitwise-OR allreduce of the whole filter (%s)" % merge_what.get(form, form),
                             "serial_ms_per_step": round(serial_ms, 4),
                             "overlap_calibration": calib,
                             "timed_step": {"overlapped": "%d build sweeps, each sweep's word range OR-allreduced on "
                                                          "a side stream while the next sweep builds" % nsw,
                                            "pipelined": "%d build sweeps, each sweep's word range OR-allreduced on "
                                                         "a side stream while the next sweep builds, the last one "
                                                         "while the next step's first sweep builds" % nsw,
                                            "serial": "build then OR-allreduce"}[mode],
                             "merge": form,
                             "merges_available": list(merges),
                             "or_allreduce_bytes_per_gpu": int(moved),
                             "or_allreduce_GBs_per_gpu": round(moved / (coll_ms * 1e-3) / 1e9, 1) if coll_ms else None}
        # Self-check (outside the timed region): one more sharded step; rank 0
        # then rebuilds the whole global key set alone, shard by shard, and
        # compares every word.  Its build time is the 1-GPU time of this same
        # workload (C5 on one GPU), for the strong-scaling curve.
        step()
        torch.cuda.synchronize(dev)
        if args.inject_merge_fault and rank == 0:
            words[nw // 3] ^= 1 << 17  # tests: a merge that lost a bit must invalidate the line
        if rank == 0:
            try:
                ref = torch.zeros_like(words)
                buf = torch.empty((nmax, 16), dtype=torch.uint8, device=dev)
                one_ms = 0.0
                for r in range(world):
                    a, b = shard(total, world, r) if scaling == "strong" else (r * npg, (r + 1) * npg)
                    ctx.gen_key16_dev(SEED_MEMBERS, a, b - a, buf[: b - a])
                    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record()
                    ctx.build_fixed_dev(buf[: b - a], 16, b - a, nb, k, ref)
                    s1.record()
                    torch.cuda.synchronize(dev)
                    one_ms += s0.elapsed_time(s1)
                ctx.sync()
                out["multi_gpu_merged_equals_single_gpu_build"] = bool(torch.equal(ref, words))
                out["single_gpu_same_workload"] = {
                    "what": "rank 0 alone builds all %d keys into the same filter (build kernels only)" % total,
                    "ms": round(one_ms, 3), "value": round(total / (one_ms * 1e-3) / 1e6, 2), "unit": "Mkeys/s"}
                del ref, buf
            except Exception as e:  # report, never lose the bench line
                out["multi_gpu_check_error"] = repr(e)[:200]
        if ipc:
            torch.cuda.synchronize(dev)
            poisoned, tmo = ipc.status()
            out["step_split"]["flag_timeouts"] = int(max_over_ranks(float(tmo)))
            out["step_split"]["merge_poisoned"] = bool(max_over_ranks(float(poisoned)))
        out["step_split"].update(merge_notes)
        if "single_gpu_same_workload" in out:
            out["speedup_vs_single_gpu_same_workload"] = round(out["single_gpu_same_workload"]["ms"] / ms, 3)
        dist.barrier()

    # Full-size parity in the bench line itself: the filter the timed steps built
    # (N = 1: C2; N > 1: the merged C5 filter on rank 0) against the oracle's
    # committed digest.  Outside the timed region.
    if rank == 0 and not args.filter_keys and scaling == "strong":
        name = {100_000_000: "c2", 1_000_000_000: "c5"}.get(total)
        if name:
            torch.cuda.synchronize(dev)
            out["words_equal_oracle_fixture"] = fixture_check(words, name, nb)
    # A line whose own checks fail publishes no number:
    # value null, the reasons listed, and a non-zero exit after the line.
    invalid = invalid_reasons(out, timed_merge=form if world > 1 else None)
    if world > 1:  # every rank exits the same way
        bad = torch.tensor([1 if invalid else 0], dtype=torch.int32, device="cpu" if host_coll else dev)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if int(bad.item()) and not invalid:
            invalid = ["a check failed on another rank"]
    if invalid:
        out["value"] = None
        out["invalid"] = invalid
    if args.verify and rank == 0 and world == 1:
        import oracle_ct
        orc = oracle_ct.load()
        host = orc.key16(SEED_MEMBERS, 0, npg)
        ref = orc.build_fixed_mt(host, 16, nb, k, 16)
        out["verified_bit_exact"] = bool(np.array_equal(words.cpu().numpy().view(np.uint64), ref))

    if not args.no_probe:
        out["probe"] = bench_probe(ctx, dev, args, world, rank, max_over_ranks)
    if world == 1 and not args.no_exact10:
        out["c2_exact_10_bits_per_key"] = bench_exact10(ctx, keys, npg)
    if world == 1 and not args.no_c1:
        out["c1_gpu"] = bench_c1_gpu(ctx, dev)
    if not args.no_e2e and rank == 0 and world == 1:
        out["e2e"] = bench_e2e(ctx, keys, npg, nb, k)

    del keys
    words = None
    torch.cuda.empty_cache()
    if not args.no_varlen and world == 1:
        out["varlen"] = bench_varlen(ctx, dev, args)
    if not args.no_c5 and world == 1:
        out["c5_shard"] = bench_c5_shard(ctx, dev)
        torch.cuda.empty_cache()
    if not args.no_c5_full and world == 1:
        out["c5_full"] = bench_c5_full(ctx, dev)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(nb, k, args.cpu_seconds)
        out["cpu_baseline"]["gpu_over_cpu_1thread"] = round(value / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        out["native"] = native_record()
        # The full record goes to a file; stdout gets ONE compact line (numbers,
        # no prose) that fits the ~8 KB of output the driver keeps, so every
        # leg — the C3 probe half of the metric included — is driver-observed.
        out["detail"] = write_detail(out, args.detail_out)
        print(json.dumps(compact_line(out), separators=(",", ":")), flush=True)
    if ipc:
        ipc.close(check=False)  # (a poisoned merge is in step_split and `invalid`)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if out.get("invalid"):
        sys.exit(3)


def invalid_reasons(out, timed_merge=None):
    """Why this line's headline number cannot stand: a failed word check, an
    error in the self-check, or (N > 1, the timed merge IPC) a poisoned merge
    or a flag wait that timed out during the timed steps."""
    why = []
    for k in ("words_equal_oracle_fixture", "multi_gpu_merged_equals_single_gpu_build", "verified_bit_exact"):
        if out.get(k) is False:
            why.append(k + " is false")
    if out.get("multi_gpu_check_error"):
        why.append("multi_gpu_check_error")
    ss = out.get("step_split") or {}
    if timed_merge == "ipc" and (ss.get("flag_timeouts") or ss.get("merge_poisoned")):
        why.append("the timed IPC merge was poisoned (%s flag waits timed out)" % ss.get("flag_timeouts"))
    return why


def write_detail(out, path):
    """The full bench record (every field, with its prose) as JSON at `path`;
    returns the path written relative to the repo, or None."""
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return os.path.relpath(path, ROOT)
    except OSError:
        return None


def _units(roof):
    """A leg's unit busy fractions from its roofline.secondary, numbers only
    (what each means: profiles/README.md, "bench line schema")."""
    sec = (roof or {}).get("secondary") or {}
    u = {k: sec[k]["frac"] for k in ("hbm_measured", "valu", "lds") if isinstance(sec.get(k), dict)}
    if isinstance(sec.get("lds"), dict) and sec["lds"].get("bank_conflict_share") is not None:
        u["lds_conflict"] = sec["lds"]["bank_conflict_share"]
    if u:
        u["limiter"] = roof.get("limiter")
    return u


def _leg_roof(roof):
    """The numbers of one leg's roofline object (no prose)."""
    if not roof:
        return None
    r = {k: roof[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms", "algorithmic_bytes")
         if k in roof}
    u = _units(roof)
    if u:
        r["units"] = u
    if roof.get("traffic_stale"):
        r["traffic_stale"] = True
    return r


def compact_line(out):
    """The one JSON line bench.py prints: the contract's fields plus every leg's
    numbers, without the prose of the full record (write_detail).  The schema is
    documented in profiles/README.md; tests/test_bench_roofline.py keeps it
    under LINE_BUDGET bytes."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    c = {k: out[k] for k in keep if k in out}
    cfg = dict(out.get("config", {}))
    ep = cfg.get("entry_point", "")
    cfg["entry_point"] = ep.split(" ")[0] if ep else ep
    c["config"] = cfg
    roof = out.get("roofline") or {}
    r = _leg_roof(roof) or {}
    for k in ("pass_a_ms", "pass_b_ms", "algorithmic_bytes_per_key", "traffic_source"):
        if k in roof:
            r[k] = roof[k]
    if "hash_walk_floor" in roof:
        hw = roof["hash_walk_floor"]
        r["hash_walk_floor_ms"] = {k: hw.get(k) for k in ("ms", "pass_a_geometry_ms", "with_claims_and_slot_writes_ms")}
        if "phase" in hw:
            r["pass_a_phase"] = {k: v for k, v in hw["phase"].items() if k != "source"}
    c["roofline"] = r
    for k in ("invalid", "words_equal_oracle_fixture", "multi_gpu_merged_equals_single_gpu_build",
              "multi_gpu_check_error", "verified_bit_exact", "speedup_vs_single_gpu_same_workload"):
        if k in out:
            c[k] = out[k]
    if "step_split" in out:
        ss = out["step_split"]
        c["step_split"] = {k: ss.get(k) for k in ("build_ms", "or_allreduce_ms", "serial_ms_per_step",
                                                  "or_allreduce_bytes_per_gpu", "or_allreduce_GBs_per_gpu",
                                                  "overlap_calibration", "timed_step", "merge", "merges_available",
                                                  "merges_agree", "ipc_error", "flag_timeouts", "merge_poisoned")}
    if "single_gpu_same_workload" in out:
        sg = out["single_gpu_same_workload"]
        c["single_gpu_same_workload"] = {"ms": sg.get("ms"), "value": sg.get("value")}
    legs = {}
    pr = out.get("probe")
    if pr:
        legs["c3_probe"] = {"ms": pr["ms"], "value": pr["value"], "unit": pr["unit"],
                            "roofline": _leg_roof(pr.get("roofline")),
                            "answers_equal_oracle_fixture": pr.get("answers_equal_oracle_fixture"),
                            "member_rows_all_hit": pr.get("member_rows_all_hit")}
        for name in ("fset", "fset_mixed", "fset_rows1"):
            f = pr.get(name)
            if f:
                legs[name] = {"ms": f["ms"], "value": f["value"], "roofline": _leg_roof(f.get("roofline"))}
                for k in ("answers_equal_oracle_fixture", "answers_equal_u64_rows"):
                    if k in f:
                        legs[name][k] = f[k]
    ex = out.get("c2_exact_10_bits_per_key")
    if ex:
        legs["c2_exact10"] = {k: ex.get(k) for k in ("value", "kernel_ms", "pass_a_ms", "pass_b_ms", "fill_ratio",
                                                     "fill_ratio_expected", "words_equal_oracle_fixture")}
        legs["c2_exact10"]["roofline"] = _leg_roof(ex.get("roofline"))
    vl = out.get("varlen")
    if vl:
        legs["c4"] = {k: vl.get(k) for k in ("value", "ms_per_step", "kernel_ms", "pass_a_ms", "pass_b_ms",
                                             "words_equal_oracle_fixture")}
        legs["c4"]["roofline"] = _leg_roof(vl.get("roofline"))
    c5 = out.get("c5_shard")
    if c5:
        legs["c5_shard"] = {k: c5.get(k) for k in ("value", "kernel_ms", "pass_a_ms", "pass_b_ms",
                                                   "words_equal_oracle_fixture")}
        legs["c5_shard"]["roofline"] = _leg_roof(c5.get("roofline"))
    c5f = out.get("c5_full")
    if c5f:
        legs["c5_full"] = {k: c5f.get(k) for k in ("value", "ms", "kernel_ms", "sweeps", "words_equal_oracle_fixture")}
        legs["c5_full"]["roofline"] = _leg_roof(c5f.get("roofline"))
    c1 = out.get("c1_gpu")
    if c1:
        legs["c1_gpu"] = {"build_ms": c1["build"]["ms"], "probe_ms": c1["probe"]["ms"],
                          "filter_equals_fixture": c1.get("filter_equals_fixture"),
                          "nonmember_answers_equal_fixture": c1.get("nonmember_answers_equal_fixture"),
                          "members_all_hit": c1.get("members_all_hit")}
    e2 = out.get("e2e")
    if e2:
        fw = e2.get("flush_walk") or {}
        sst = e2.get("sst_flush_latency") or []
        legs["e2e"] = {"pageable_ms": e2["pageable"]["ms"], "pinned_ms": e2["pinned"]["ms"], "value": e2["value"],
                       "pcie_GBs": e2["pageable"]["pcie_GBs"],
                       "crc32_ms": (e2.get("with_crc32") or {}).get("ms"),
                       "crc_equals_zlib": (e2.get("with_crc32") or {}).get("crc_equals_zlib"),
                       "flush_walk": {k: fw.get(k) for k in ("keys", "walk_ms", "stream_ms", "host_insert_1t_ms",
                                                             "bit_exact", "error") if k in fw},
                       "sst_flush_keys_ms_gpu_ms_cpu_ms": [[x["keys"], x["ms"], x["gpu_ms"], x["cpu_oracle_1t_ms"]]
                                                           for x in sst],
                       "sst_flush_bit_exact": all(x.get("bit_exact") for x in sst) if sst else None,
                       "host_max_keys": e2.get("host_max_keys")}
    if legs:
        c["legs"] = legs
    cb = out.get("cpu_baseline")
    if cb:
        cc = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "cpu", "gpu_over_cpu_1thread")}
        cc["sample"] = "first %s C2 keys into the full C2 filter, 1 thread, oracle/bloom_oracle.c -O3 -march=native" \
            % cb.get("sample", "").split(" ")[1] if cb.get("sample") else None
        mt = cb.get("multi_thread") or {}
        cc["multi_thread"] = {"value": mt.get("value"), "cores": mt.get("cores")}
        c1c = cb.get("c1") or {}
        cc["c1_Mkeys_s"] = {k: (c1c.get(k) or {}).get("value") for k in ("build_1t", "probe_1t", "build_mt", "probe_mt")}
        c["cpu_baseline"] = cc
    nat = out.get("native")
    if nat:
        c["native"] = {k: nat.get(k) for k in ("library", "kernel_sources_sha", "library_sha256_16", "gcn_arch")}
    for k in ("detail",):
        if out.get(k):
            c[k] = out[k]
    return c


LINE_BUDGET = 6000  # bytes: the driver keeps ~8 KB of stdout + stderr


def bench_c1_gpu(ctx, dev, reps=20):
    """C1's workload (configs[0]: build new(100000, 0.01) from 100 k key16
    members, probe 100 k members + 100 k non-members) on the GPU, device-
    resident keys, next to cpu_baseline.c1; the filter and the non-member
    answers against the committed C1 fixture (tests/golden/c1_fixture.json)."""
    import hashlib
    import json

    import numpy as np
    import torch

    import lsmbloom
    n = 100_000
    nb, k = lsmbloom.params(n, 0.01)
    mem = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    non = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(SEED_MEMBERS, 0, n, mem)
    ctx.gen_key16_dev(SEED_FRESH, 0, n, non)
    w = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    q = torch.cat([mem, non])
    out = torch.zeros((2 * n, 1), dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(3):
        ctx.build_fixed_dev_new(mem, 16, n, nb, k, w)
        ctx.probe_dev([(w, nb, k)], q, 2 * n, out, key_len=16)
    torch.cuda.synchronize(dev)
    ev[0].record()
    for _ in range(reps):
        ctx.build_fixed_dev_new(mem, 16, n, nb, k, w)
    ev[1].record()
    ev[2].record()
    for _ in range(reps):
        ctx.probe_dev([(w, nb, k)], q, 2 * n, out, key_len=16)
    ev[3].record()
    torch.cuda.synchronize(dev)
    b_ms, p_ms = ev[0].elapsed_time(ev[1]) / reps, ev[2].elapsed_time(ev[3]) / reps
    res = {"workload": "C1 (configs[0]) on the GPU: build new(%d, 0.01) (%d bits, k=%d) from %d key16 members "
                       "(lsmb_build_fixed_dev_new), probe %d members + %d non-members" % (n, nb, k, n, n, n),
           "build": {"ms": round(b_ms, 4), "value": round(n / (b_ms * 1e-3) / 1e6, 1), "unit": "Mkeys/s",
                     "strategy": lsmbloom.build_strategy(nb, n, k)},
           "probe": {"ms": round(p_ms, 4), "value": round(2 * n / (p_ms * 1e-3) / 1e6, 1), "unit": "Mkeys/s"}}
    p = os.path.join(ROOT, "tests", "golden", "c1_fixture.json")
    if os.path.exists(p):
        fx = json.load(open(p))
        hw = w.cpu().numpy().view(np.uint64)
        blk = np.concatenate([np.array([k, nb, hw.size], dtype="<u4").view(np.uint8), hw.astype("<u8").view(np.uint8)])
        m = out[n:].cpu().numpy().reshape(-1)
        res["filter_equals_fixture"] = hashlib.sha256(blk.tobytes()).hexdigest() == fx["serialized_sha256"]
        res["nonmember_answers_equal_fixture"] = hashlib.sha256(m.tobytes()).hexdigest() == fx["nonmember_probe_sha256"]
        res["members_all_hit"] = bool(out[:n].bool().all().item())
    return res


def bench_exact10(ctx, keys, n, reps=10):
    """C2's exact 10-bits-per-key variant: num_bits =
    10 n, k = 7 (reachable in the reference through deserialize of a zeroed
    header + inserts, src/bloom/mod.rs:123-168), same keys, device build."""
    import numpy as np
    import torch

    import lsmbloom
    nb, k = 10 * n, 7
    if nb >= 2 ** 32:
        return {"skipped": "10 n >= 2^32 bits is not representable (num_bits is u32)"}
    w = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=keys.device)
    ctx.set_timing(True)
    kt = np.zeros(3)
    for i in range(reps + 2):
        ctx.build_fixed_dev_new(keys, 16, n, nb, k, w)
        ctx.sync()
        torch.cuda.synchronize(keys.device)
        if i >= 2:
            kt += np.array(ctx.last_build_ms())
    ctx.set_timing(False)
    kt /= reps
    alg = 16 * n + 8 * lsmbloom.num_words(nb)
    fill = int(np.bitwise_count(w.cpu().numpy().view(np.uint64)).sum(dtype=np.uint64))
    res = {"workload": "C2 exact: %d 16-B keys into num_bits = 10 n = %d, k = 7" % (n, nb),
           "value": round(n / (kt[0] * 1e-3) / 1e6, 1), "unit": "Mkeys/s", "kernel_ms": round(float(kt[0]), 4),
           "pass_a_ms": round(float(kt[1]), 4), "pass_b_ms": round(float(kt[2]), 4),
           "strategy": lsmbloom.build_strategy(nb, n, k),
           "frac": round(alg / (kt[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "roofline": leg_roofline("exact10" if n == 100_000_000 else None, alg, kt[0],
                                    "build (k_bin + k_apply + k_ovf_apply)")}
    # expected fill of an ideal filter: 1 - exp(-k n / m)
    res["fill_ratio"] = round(fill / nb, 5)
    res["fill_ratio_expected"] = round(1 - float(np.exp(-k * n / nb)), 5)
    if n == 100_000_000:
        res["words_equal_oracle_fixture"] = fixture_check(w, "c2_exact10", nb)
    del w
    return res


def bench_c5_shard(ctx, dev, reps=10):
    """configs[4]'s per-GPU build on one GPU: the first 125 M C5 keys (shard 0
    of 8) into new(1e9, 0.01) = 2^32-1 bits, fresh, device-resident keys
    generated on the device; every word against the oracle's digest
    (tests/golden/fullsize_fixture.json "c5_shard0")."""
    import numpy as np
    import torch

    import lsmbloom
    n = 125_000_000
    nb, k = lsmbloom.params(1_000_000_000, 0.01)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(SEED_MEMBERS, 0, n, keys)
    w = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    ctx.set_timing(True)
    kt = np.zeros(3)
    for i in range(reps + 2):
        ctx.build_fixed_dev_new(keys, 16, n, nb, k, w)
        ctx.sync()
        torch.cuda.synchronize(dev)
        if i >= 2:
            kt += np.array(ctx.last_build_ms())
    ctx.set_timing(False)
    kt /= reps
    alg = 16 * n + 8 * lsmbloom.num_words(nb)
    res = {"workload": "C5 shard 0 of 8: %d 16-B keys into new(1e9, 0.01) = %d bits, k = %d" % (n, nb, k),
           "value": round(n / (kt[0] * 1e-3) / 1e6, 1), "unit": "Mkeys/s", "kernel_ms": round(float(kt[0]), 4),
           "pass_a_ms": round(float(kt[1]), 4), "pass_b_ms": round(float(kt[2]), 4),
           "strategy": lsmbloom.build_strategy(nb, n, k),
           "roofline": leg_roofline("c5", alg, kt[0], "build (2 sweeps of k_bin + k_apply<21> + k_ovf_apply)")}
    res["words_equal_oracle_fixture"] = fixture_check(w, "c5_shard0", nb)
    del w, keys
    return res


def bench_c5_full(ctx, dev, reps=4):
    """configs[4]'s whole run on ONE GPU: all 1e9 C5 keys into new(1e9, 0.01) =
    2^32-1 bits, built the way each rank builds its shard at N > 1 (fresh,
    sweep by sweep: lsmb_build_fixed_dev_sweep_new), device-resident keys
    generated on the device, every word against the oracle's digest
    (tests/golden/fullsize_fixture.json "c5").  The 1-GPU point of the N > 1
    strong-scaling curve, whose lines time the same workload split N ways."""
    import numpy as np
    import torch

    import lsmbloom
    n = 1_000_000_000
    nb, k = lsmbloom.params(n, 0.01)
    keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    ctx.gen_key16_dev(SEED_MEMBERS, 0, n, keys)
    w = torch.empty(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
    nsw = lsmbloom.build_sweeps(nb, n, k)

    def build():
        for s in range(nsw):
            ctx.build_fixed_dev_sweep_new(keys, 16, n, nb, k, w, s)
    build()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        build()
    ev[1].record()
    torch.cuda.synchronize(dev)
    ms = ev[0].elapsed_time(ev[1]) / reps
    alg = 16 * n + 8 * lsmbloom.num_words(nb)
    res = {"workload": "C5 (configs[4]) on one GPU: %d 16-B keys into new(1e9, 0.01) = %d bits, k = %d, %d sweeps "
                       "(lsmb_build_fixed_dev_sweep_new, as each rank at N > 1)" % (n, nb, k, nsw),
           "value": round(n / (ms * 1e-3) / 1e6, 1), "unit": "Mkeys/s", "ms": round(ms, 3), "kernel_ms": round(ms, 3),
           "sweeps": nsw, "strategy": lsmbloom.build_strategy(nb, n, k),
           "roofline": leg_roofline("c5_full", alg, ms, "build (%d sweeps of k_bin + k_apply<21> + k_ovf_apply)" % nsw)}
    res["words_equal_oracle_fixture"] = fixture_check(w, "c5", nb)
    del w, keys
    return res


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
    # the same flush with the block's CRC-32 computed on the device words
    # (lsmb_build_block_crc), pinned keys
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _, crc = ctx.build_block_crc(src, nb, k, key_len=16, out=block)
        ts.append(time.perf_counter() - t0)
    import zlib
    res["with_crc32"] = {"ms": round(float(np.median(ts)) * 1e3, 2),
                         "crc_equals_zlib": zlib.crc32(block) == crc}
    # SST-sized flushes: one lsmb_build_block call per table, sized like
    # SSTableBuilder::with_estimated_keys (builder.rs:74); latency per call
    # (H2D, kernels, D2H, sync) next to the 1-thread CPU oracle on the same
    # keys.  Each size runs twice: through the default dispatch ("path": the
    # library's host loop at or below lsmb_host_max_keys, else the GPU) and
    # forced onto the GPU (threshold 0): the crossover sets the threshold.
    import oracle_ct
    orc = oracle_ct.load()
    small = []
    thr = lsmbloom.host_max_keys()

    def lat(ks, nb_m, k_m, blk, reps=20):
        ctx.build_block(ks, nb_m, k_m, key_len=16, out=blk)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ctx.build_block(ks, nb_m, k_m, key_len=16, out=blk)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    for m in (250, 500, 1000, 2000, 4000, 8000, 100_000, 1_000_000):
        nb_m, k_m = lsmbloom.params(m, 0.01)
        ks = np.ascontiguousarray(host[: m * 16])
        blk = np.empty(lsmbloom.serialized_size(nb_m), dtype=np.uint8)
        t_default = lat(ks, nb_m, k_m, blk)
        lsmbloom.set_host_max_keys(0)
        blk_gpu = np.empty_like(blk)
        t_gpu = lat(ks, nb_m, k_m, blk_gpu)
        lsmbloom.set_host_max_keys(thr)
        t0 = time.perf_counter()
        ref = orc.build_fixed(ks.reshape(m, 16), 16, nb_m, k_m)
        tc = time.perf_counter() - t0
        small.append({"keys": m, "path": "host" if m <= thr else lsmbloom.build_strategy(nb_m, m, k_m),
                      "ms": round(t_default, 4), "gpu_ms": round(t_gpu, 4), "cpu_oracle_1t_ms": round(tc * 1e3, 4),
                      "bit_exact": bool(np.array_equal(np.frombuffer(blk[12:].tobytes(), dtype=np.uint64), ref)
                                        and np.array_equal(blk, blk_gpu))})
    res["host_max_keys"] = thr
    # Flush-shaped end to end from a host structure: a C++
    # driver walks an ordered memtable of 4 M 16-B keys and feeds every key to
    # lsmb_stream_add (chunks upload and build while the walk goes on), then
    # lsmb_stream_finish_block; beside it the same walk through the library's
    # per-key host insert + serialize (the reference's flush, one thread).
    import subprocess
    exe = os.path.join(ROOT, "storage-engine_amd", "build", "flush_e2e")
    try:
        r = subprocess.run([exe, "4000000"], capture_output=True, text=True, timeout=180)
        res["flush_walk"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
            {"error": (r.stdout + r.stderr)[-300:]}
    except Exception as e:  # report, never lose the bench line
        res["flush_walk"] = {"error": repr(e)[:200]}
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

    def build():
        if args.accumulate:
            words.zero_()
            ctx.build_var_dev(data, offs, n, nb, k, words)
        else:
            ctx.build_var_dev_new(data, offs, n, nb, k, words)

    def step():
        build()

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
        build()
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
           "strategy": lsmbloom.build_strategy(nb, n),
           "roofline": leg_roofline("c4" if n == 100_000_000 else None, alg, kt[0],
                                    "build (k_hash_var + k_bin<Recs> + k_apply + k_ovf_apply)")}
    if n == 100_000_000:
        res["words_equal_oracle_fixture"] = fixture_check(words, "c4", nb)
    del data, offs, words
    torch.cuda.empty_cache()
    return res


KERNEL_SOURCES = ("storage-engine_amd/csrc/bloom_build.hip", "storage-engine_amd/csrc/bloom_probe.hip",
                  "storage-engine_amd/csrc/kernels.hpp", "storage-engine_amd/csrc/bloom_math.hpp",
                  "storage-engine_amd/csrc/xxh3.hpp", "storage-engine_amd/csrc/keysrc.hpp",
                  "storage-engine_amd/csrc/hash_var.hpp")


def build_sources_sha():
    """sha256 over the build and probe kernels' sources: stamps profiles/traffic.json."""
    import hashlib
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def committed_legs():
    """Per-leg PMC figures from the committed rocprofv3 summary
    (profiles/traffic.json, tools/profile_legs.sh + tools/prof_summary.py
    --legs: every leg in a process of its own, separate FETCH_SIZE /
    WRITE_SIZE / SQ passes, FETCH_SIZE doubled per the gfx950 note in
    MI355X_MICROARCH.md).  `fresh` is False when the kernels' sources changed
    since that profile (its stamped sha differs)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    t = json.load(open(p))
    if t.get("format") != 2:
        return None
    return {"legs": t["legs"], "source": "%s (%s)" % (os.path.relpath(p, ROOT), t.get("profile")),
            "fresh": t.get("kernel_src_sha") == build_sources_sha()}


# Ceilings of the secondary units, per profiled launch (clock-independent: the
# launch's own cycles from GRBM_GUI_ACTIVE, summed over the 8 XCDs).
# VALU: a wave64 instruction occupies its SIMD ~4 cycles (tools/mb_valu.hip,
# profiles/r04/r04b_valu_issue.jsonl: 4.1-4.7 for the multiplies, converts,
# f64, min, bfe and 64-bit ops; 2.3-2.5 for add / xor / mul_f32), 1024 SIMDs.
# LDS: SQ_LDS_IDX_ACTIVE = LDS-array cycles over the 256 CUs' LDS.
VALU_CYCLES_PER_INST = 4.0
SATURATED = 0.75  # a unit busier than this fraction of the launch's cycles is its limiter
# The C2 compute floor (tools/mb_hash.hip, profiles/r06/r06c_hash_floor.log): XXH3-128
# of 100 M 16-B keys + their 7 exact positions, k = 7 unrolled, at full
# occupancy; the same at pass A's geometry (1024-thread workgroups, one per CU),
# and with pass A's claims and ring slot writes added (no flush, no barriers).
HASH_WALK_FLOOR = {"ms": 0.363, "pass_a_geometry_ms": 0.428, "with_claims_and_slot_writes_ms": 0.558,
                   "source": "profiles/r06/r06c_hash_floor.log",
                   "what": "no build can beat the hash + position arithmetic alone"}
# Where pass A's phase goes (LSMB_STAMP build, profiles/r06/r06c_stamps.log;
# shares of the cycles per phase per wave) and the ablations around it
# (tools/build_variants.sh + run_variants.sh, profiles/r06/r06c_passA_ablations.log:
# pass A ms with no flush / no region stores / every region store dropped).
PASS_A_PHASE = {"cycles": 6241, "work": 0.356, "barrier1": 0.170, "flush": 0.321, "barrier2": 0.154,
                "ablation_pass_a_ms": {"product": 0.982, "no_flush": 0.582, "no_region_stores": 0.739,
                                       "stores_dropped": 0.864},
                "source": "profiles/r06/r06c_stamps.log, r06c_passA_ablations.log"}


def native_record():
    """What ran: the HIP library this process loaded (path, size, sha256 prefix),
    the device it opened, the kernels' source sha, and the strategies the C2 /
    C3 legs dispatched — so a bench line can be tied to native code."""
    import hashlib

    import lsmbloom
    rec = {"library": os.path.relpath(lsmbloom.LIB_PATH, ROOT), "kernel_sources_sha": build_sources_sha()}
    try:
        with open(lsmbloom.LIB_PATH, "rb") as f:
            blob = f.read()
        rec["library_bytes"] = len(blob)
        rec["library_sha256_16"] = hashlib.sha256(blob).hexdigest()[:16]
    except OSError as e:
        rec["library_error"] = repr(e)[:120]
    try:
        import torch
        rec["device"] = torch.cuda.get_device_name(torch.cuda.current_device())
        rec["gcn_arch"] = getattr(torch.cuda.get_device_properties(torch.cuda.current_device()), "gcnArchName", None)
    except Exception as e:  # never lose the bench line
        rec["device_error"] = repr(e)[:120]
    rec["abi_version"] = int(lsmbloom.lib().lsmb_abi_version())
    rec["c2_build_strategy"] = lsmbloom.build_strategy(956715292, 100_000_000)
    return rec


def leg_roofline(leg, alg_bytes, kernel_ms, kernel, legs=None):
    """roofline object of one bench leg: algorithmic HBM bytes per launch over
    the launch's kernel time (HIP events) against 8 TB/s; `traffic` = HBM
    bytes per launch from the committed PMC passes; `secondary` = how busy the
    VALU and the LDS were in the profiled launch, and `limiter` = the busiest
    of HBM (measured traffic), VALU and LDS."""
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kernel,
            "algorithmic_bytes": int(alg_bytes), "kernel_ms": round(float(kernel_ms), 4)}
    legs = legs if legs is not None else committed_legs()
    if not legs or leg not in legs["legs"]:
        return roof
    roof["traffic_source"] = legs["source"]
    if not legs["fresh"]:
        roof["traffic_stale"] = "kernel sources changed since %s was profiled" % legs["source"]
        return roof
    p = legs["legs"][leg]["per_launch"]
    roof["traffic"] = p.get("hbm_bytes")
    cyc = p.get("grbm_gui_active", 0) / 8.0
    prof_us = p.get("kernel_us")
    sec = {}
    if prof_us:
        sec["hbm_measured"] = {"achieved": round(p["hbm_bytes"] / (prof_us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(p["hbm_bytes"] / (prof_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                               "what": "PMC traffic over the profiled launch's kernel time"}
    if cyc > 0 and p.get("valu_insts"):
        sec["valu"] = {"insts_per_launch": p["valu_insts"], "cycles_per_inst": VALU_CYCLES_PER_INST,
                       "frac": round(p["valu_insts"] * VALU_CYCLES_PER_INST / (1024 * cyc), 4),
                       "what": "wave64 VALU instructions x 4 cycles / (1024 SIMDs x the launch's cycles)"}
    if cyc > 0 and p.get("lds_idx_active") is not None:
        la = p["lds_idx_active"]
        sec["lds"] = {"array_cycles_per_launch": la, "frac": round(la / (256 * cyc), 4),
                      "bank_conflict_share": round(p.get("lds_bank_conflict", 0) / la, 4) if la else None,
                      "insts_per_launch": p.get("lds_insts"),
                      "issue_est_frac": round(p.get("lds_insts", 0) * 10.1 / (256 * cyc), 4),
                      "what": "SQ_LDS_IDX_ACTIVE (LDS-array cycles) / (256 CUs x the launch's cycles); "
                              "issue_est: SQ_INSTS_LDS x 10.1 cycles (ds_add_rtn, tools/mb_lds.hip)"}
    if sec:
        sec["launch_cycles"] = int(cyc)
        roof["secondary"] = sec
        cand = {k: v["frac"] for k, v in sec.items() if isinstance(v, dict) and "frac" in v}
        if cand:
            # A unit is named the limiter only when it is near saturation; a
            # launch whose busiest unit sits well below that is bound by latency
            # and synchronisation (pass A's barrier-separated phases), not by it.
            roof["busiest"] = max(cand, key=cand.get)
            roof["limiter"] = roof["busiest"] if cand[roof["busiest"]] >= SATURATED else "none"
    return roof


def fixture_check(words, name, num_bits):
    """Every word of a full-size filter against the oracle's digest committed in
    tests/golden/fullsize_fixture.json (tests/golden/gen_fullsize.py): True /
    False, or None when this run's configuration is not the fixture's."""
    import hashlib
    import json

    import numpy as np
    p = os.path.join(ROOT, "tests", "golden", "fullsize_fixture.json")
    if not os.path.exists(p):
        return None
    fx = json.load(open(p)).get(name)
    if not fx or fx["num_bits"] != num_bits:
        return None
    w = np.ascontiguousarray(words.cpu().numpy().view(np.uint64), dtype="<u8")
    return bool(w.size == fx["words"] and int(np.bitwise_count(w).sum()) == fx["popcount"]
                and hashlib.sha256(w.tobytes()).hexdigest() == fx["sha256"])


class ProbeLegs:
    """C3's data (configs[2]) and its three device probes, shared by
    bench_probe and tools/legs.py (rocprofv3 passes per leg): F per-SSTable
    filters sized like SSTableBuilder::new (1000 keys, 0.01) and Q lookup keys
    (50 % members drawn across the F filters, 50 % fresh).
      probe()       lsmb_probe_dev over the F filters (k_probe_sliced)
      fset()        lsmb_fset_probe_dev, the same F tables with their key ranges
      fset_mixed()  a set of two sizes: F/2 of them + F/2 x new(4000, 0.01)"""

    def __init__(self, ctx, dev, Q, F):
        import numpy as np
        import torch

        import lsmbloom
        self.ctx, self.dev, self.Q, self.F = ctx, dev, Q, F
        nb, k = lsmbloom.params(1000, 0.01)
        self.nb, self.k = nb, k
        nw = lsmbloom.num_words(nb)
        self.filt = []
        self.members = torch.empty((F * 1000, 16), dtype=torch.uint8, device=dev)
        for f in range(F):
            ctx.gen_key16_dev(0xF000 + f, 0, 1000, self.members[f * 1000:(f + 1) * 1000])
            w = torch.zeros(nw, dtype=torch.int64, device=dev)
            ctx.build_fixed_dev(self.members[f * 1000:(f + 1) * 1000], 16, 1000, nb, k, w)
            self.filt.append((w, nb, k))
        self.q = torch.empty((Q, 16), dtype=torch.uint8, device=dev)
        ctx.gen_key16_dev(SEED_FRESH, 0, Q, self.q)
        g = torch.Generator(device="cpu").manual_seed(1)
        self.sel = torch.randint(0, F * 1000, (Q // 2,), generator=g).to(dev)
        self.q[: Q // 2] = self.members[self.sel]
        self.out = torch.zeros((Q, (F + 7) // 8), dtype=torch.uint8, device=dev)
        self.fout = torch.zeros(Q, dtype=torch.int64, device=dev)
        self.fout1 = torch.zeros(Q, dtype=torch.uint8, device=dev)
        # the same F tables as a filter set, with their key ranges
        self.fs = lsmbloom.FilterSet(ctx)
        self.slots = []
        for f in range(F):
            rows = self.members[f * 1000:(f + 1) * 1000].cpu().numpy()
            srt = sorted(bytes(r) for r in rows)
            self.slots.append(self.fs.add_filter(
                lsmbloom.BloomFilter(self.filt[f][0].cpu().numpy().view(np.uint64), k, nb), srt[0], srt[-1]))
        # mixed sizes: F/2 of the C3 tables + F/2 compaction-sized new(4000, 0.01)
        # (38 271 bits): two (num_bits, k) classes, each its own LDS table
        self.fsm = lsmbloom.FilterSet(ctx)
        nb4, k4 = lsmbloom.params(4000, 0.01)
        big = torch.empty((4000, 16), dtype=torch.uint8, device=dev)
        for f in range(F):
            if f < F // 2:
                rows = self.members[f * 1000:(f + 1) * 1000].cpu().numpy()
                bf = lsmbloom.BloomFilter(self.filt[f][0].cpu().numpy().view(np.uint64), k, nb)
            else:
                ctx.gen_key16_dev(0xF100 + f, 0, 4000, big)
                w4 = torch.zeros(lsmbloom.num_words(nb4), dtype=torch.int64, device=dev)
                ctx.build_fixed_dev(big, 16, 4000, nb4, k4, w4)
                rows = big.cpu().numpy()
                bf = lsmbloom.BloomFilter(w4.cpu().numpy().view(np.uint64), k4, nb4)
            srt = sorted(bytes(r) for r in rows)
            self.fsm.add_filter(bf, srt[0], srt[-1])
        self.nw = nw

    def probe(self):
        self.ctx.probe_dev(self.filt, self.q, self.Q, self.out, key_len=16)

    def fset(self):
        self.fs.probe_dev(self.q, self.Q, self.fout, key_len=16)

    def fset_mixed(self):
        self.fsm.probe_dev(self.q, self.Q, self.fout, key_len=16)

    def fset_rows1(self):  # the same set, one-byte answer rows (its 8 slots fit them)
        self.fs.probe_dev(self.q, self.Q, self.fout1, key_len=16, row_bytes=1)

    def alg_bytes(self, leg):
        """Algorithmic HBM bytes of one launch: the keys, the answers and the filters."""
        if leg == "probe":
            return self.Q * 16 + self.Q * self.out.shape[1] + self.F * (12 + 8 * self.nw)
        if leg == "fset_rows1":
            return self.Q * 16 + self.Q + self.F * (12 + 8 * self.nw)
        return self.Q * 16 + self.Q * 8 + self.F * (12 + 8 * self.nw)

    def close(self):
        self.fs.close()
        self.fsm.close()


def timed_ms(fn, warmup, steps, warm_ms=0.0, min_timed_ms=0.0):
    """Average ms of fn() over `steps` calls (HIP events on the current stream).
    warm_ms / min_timed_ms: keep warming up until that much device time has
    run, and time at least that many ms of calls: a ~50 us probe needs ~20 ms
    of back-to-back work before the GPU's clock has ramped (rocprofv3: the
    C3 kernel takes 50 us in the first calls, 45.7 us from about the third
    ms on), which the legs' few warmup calls do not give it."""
    import time

    import torch
    for _ in range(max(1, warmup)):
        fn()
    torch.cuda.synchronize()
    if warm_ms > 0:
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < warm_ms:
            for _ in range(8):
                fn()
            torch.cuda.synchronize()
    if min_timed_ms > 0:
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        one = max((time.perf_counter() - t0) * 1e3, 1e-3)
        steps = max(steps, int(min_timed_ms / one) + 1)
    st = torch.cuda.Event(enable_timing=True)
    en = torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(steps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / steps


def bench_probe(ctx, dev, args, world=1, rank=0, max_over_ranks=lambda x: x):
    """C3: Q lookup keys (50% members drawn across the F filters, 50% fresh)
    against F per-SSTable filters sized like SSTableBuilder::new (1000 keys, 0.01).
    N > 1: the filters are replicated and the queries partitioned (no
    collective); the rate counts all ranks' queries over the slowest rank."""
    import torch

    F, Q_all = args.probe_filters, args.probe_keys
    Q = Q_all // world
    P = ProbeLegs(ctx, dev, Q, F)
    ms = max_over_ranks(timed_ms(P.probe, args.warmup, args.steps, warm_ms=20, min_timed_ms=10))
    alg = P.alg_bytes("probe")
    hits = int((P.out[: Q // 2] != 0).all(dim=1).sum().item())
    res = {"workload": "C3 (configs[2]): %d 16-B keys x %d filters new(1000, 0.01) (%d bits, k=%d)%s"
                       % (Q_all, F, P.nb, P.k, ", %d per GPU" % Q if world > 1 else ""),
           "value": round(Q * world / (ms * 1e-3) / 1e6, 2), "unit": "Mkeys/s", "ms": round(ms, 4),
           "achieved_GBs": round(alg / (ms * 1e-3) / 1e9, 1), "algorithmic_bytes": alg,
           "member_rows_all_hit": hits == Q // 2,
           "roofline": leg_roofline("probe" if (Q, F) == (10_000_000, 8) else None, alg, ms, "k_probe_sliced")}
    # Every answer of the full-size run against the oracle's (digests committed
    # in tests/golden/c3_fixture.json by gen_c3_fixture.py; outside the timing).
    c3fx = c3_fixture() if world == 1 else None
    if c3fx and c3fx["Q"] == Q and c3fx["F"] == F:
        res["answers_equal_oracle_fixture"] = _sha(P.out) == c3fx["probe_mask_sha256"]
    # The same batch through the device-resident filter set (lsmb_fset): per
    # key and SSTable, min_key <= key <= max_key && may_contain — the checks
    # SSTable::get makes (src/sstable/reader.rs:192-199) — for all 8 tables.
    fms = max_over_ranks(timed_ms(P.fset, args.warmup, args.steps, warm_ms=20, min_timed_ms=10))
    # a member row's own table must answer 1 (range and bloom); here sel // 1000
    own = (P.fout[: Q // 2] >> torch.tensor(P.slots, device=dev)[P.sel // 1000]) & 1
    res["fset"] = {"what": "lsmb_fset_probe_dev: range pre-check + bloom, %d tables, u64 mask per key" % F,
                   "value": round(Q * world / (fms * 1e-3) / 1e6, 2), "unit": "Mkeys/s", "ms": round(fms, 4),
                   "algorithmic_bytes": P.alg_bytes("fset"), "member_rows_own_table_hit": bool(own.all().item()),
                   "roofline": leg_roofline("fset" if (Q, F) == (10_000_000, 8) else None, P.alg_bytes("fset"), fms,
                                            "k_fset_sliced")}
    if c3fx and c3fx["Q"] == Q and c3fx["F"] == F:
        res["fset"]["answers_equal_oracle_fixture"] = _sha(P.fout) == c3fx["fset_mask_sha256"]
    # The same set with one-byte answer rows (lsmb_fset_probe_dev_rows; its 8
    # slots fit a byte): every row equal to the u64 row's low byte just made.
    u64_rows = P.fout.clone()
    r1ms = max_over_ranks(timed_ms(P.fset_rows1, args.warmup, args.steps, warm_ms=20, min_timed_ms=10))
    res["fset_rows1"] = {"what": "lsmb_fset_probe_dev_rows: the same %d-table set, one-byte answer rows" % F,
                         "value": round(Q * world / (r1ms * 1e-3) / 1e6, 2), "unit": "Mkeys/s", "ms": round(r1ms, 4),
                         "algorithmic_bytes": P.alg_bytes("fset_rows1"),
                         "answers_equal_u64_rows": bool(torch.equal(P.fout1, (u64_rows & 0xFF).to(torch.uint8))),
                         "roofline": leg_roofline("fset_rows1" if (Q, F) == (10_000_000, 8) else None,
                                                  P.alg_bytes("fset_rows1"), r1ms, "k_fset_sliced")}
    del u64_rows
    mms = max_over_ranks(timed_ms(P.fset_mixed, args.warmup, args.steps, warm_ms=20, min_timed_ms=10))
    res["fset_mixed"] = {"what": "lsmb_fset_probe_dev, %d tables of two sizes: %d x new(1000, 0.01) + %d x "
                                 "new(4000, 0.01), one LDS table per size class" % (F, F // 2, F - F // 2),
                         "value": round(Q * world / (mms * 1e-3) / 1e6, 2), "unit": "Mkeys/s", "ms": round(mms, 4),
                         "algorithmic_bytes": P.alg_bytes("fset_mixed"),
                         "roofline": leg_roofline("fset_mixed" if (Q, F) == (10_000_000, 8) else None,
                                                  P.alg_bytes("fset_mixed"), mms, "k_fset_classes")}
    if c3fx and c3fx["Q"] == Q and c3fx["F"] == F:
        res["fset_mixed"]["answers_equal_oracle_fixture"] = _sha(P.fout) == c3fx["fset_mixed_mask_sha256"]
    P.close()
    return res


def c3_fixture():
    p = os.path.join(ROOT, "tests", "golden", "c3_fixture.json")
    return json.load(open(p)) if os.path.exists(p) else None


def _sha(t):
    """sha256 of a device tensor's bytes (little-endian, row-major)."""
    import hashlib
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()


if __name__ == "__main__":
    main()
