#!/usr/bin/env python3
"""Condense a tools/profile.sh output directory into a markdown summary.

Usage: tools/prof_summary.py gpurun_out/prof_<tag> > profiles/<tag>.md
FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE is doubled (gfx950 tallies a
wide coalesced stream's 128-B requests at 64 B: MI355X_MICROARCH.md §HBM).
"""
import collections
import csv
import os
import sys


def short(name):
    n = name.replace("lsmb::(anonymous namespace)::", "").replace("lsmb::", "").replace("void ", "")
    n = n.split("(")[0]
    return n[:90]


def traffic_json(d, out):
    """Per-dispatch HBM bytes and VALU instructions of the C2 build kernels
    (pass A k_bin <Fixed16...> + pass B k_apply) -> JSON read by
    bench.py (roofline.traffic, roofline.secondary)."""
    import json
    per = collections.defaultdict(dict)
    for sub, cns in (("fetch", ("FETCH_SIZE",)), ("write", ("WRITE_SIZE",)), ("sq2", ("SQ_INSTS_VALU",))):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] in cns:
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for kn, cv in vals.items():
            for cn, v in cv.items():
                per[kn][cn] = sum(v) / len(v)
    kern = {}
    for kn, m in per.items():
        if kn.startswith(("k_bin<ks::Fixed16", "k_apply", "k_ovf_apply")):
            kern[kn] = {"read_bytes": int(2 * m.get("FETCH_SIZE", 0) * 1024),
                        "write_bytes": int(m.get("WRITE_SIZE", 0) * 1024),
                        "valu_insts": int(m.get("SQ_INSTS_VALU", 0))}
    tot = sum(v["read_bytes"] + v["write_bytes"] for v in kern.values())
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # the sha of the build kernels' sources this profile measured
    json.dump({"profile": os.path.basename(d.rstrip("/")), "build_bytes": tot, "kernels": kern,
               "build_valu_insts": sum(v["valu_insts"] for v in kern.values()),
               "kernel_src_sha": bench.build_sources_sha(),
               "note": "FETCH_SIZE x2 (gfx950), KiB -> B; mean per dispatch over separate --pmc passes"},
              open(out, "w"), indent=1)


def main(d):
    print("# rocprofv3 summary: %s\n" % os.path.basename(d.rstrip("/")))
    for sub, title in (("stats", "C2 bench"), ("stats_c5", "C5 shard: 125 M keys into 2^32-1 bits"),
                       ("stats_c4", "C4 var-len build")):
        ks = os.path.join(d, sub, "run_kernel_stats.csv")
        if not os.path.exists(ks):
            continue
        print("## Kernel time, %s (rocprofv3 --kernel-trace --stats)\n" % title)
        print("| kernel | calls | avg us | total % |")
        print("|---|---|---|---|")
        for r in csv.DictReader(open(ks)):
            print("| %s | %s | %.2f | %.1f |" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                float(r["Percentage"])))
        print()
    for sub in ("fetch_c5", "write_c5"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        print("## C5 shard, %s (mean per dispatch)\n" % sub.split("_")[0].upper())
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for kn, v in sorted(vals.items()):
            if kn.startswith(("k_bin", "k_apply")):
                m = sum(v) / len(v)
                mb = (2 if sub.startswith("fetch") else 1) * m * 1024 / 1e6
                print("- %s: %s = %.4g -> %.1f MB%s" % (kn, sub.split("_")[0].upper() + "_SIZE", m, mb,
                                                       " (x2, gfx950)" if sub.startswith("fetch") else ""))
        print()
    pmc(d, ("fetch", "write", "sq1", "sq2"), "PMC counters, C2 bench (mean per dispatch)")
    pmc(d, ("sq1_c5", "sq2_c5"), "PMC counters, C5 shard (mean per dispatch)")


def pmc(d, subs, title):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in subs:
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if agg:
        print("## %s\n" % title)
        for kn, cs in sorted(agg.items()):
            if not any(x in kn for x in ("k_", "lsmb")):
                continue
            m = {c: sum(v) / len(v) for c, v in cs.items()}
            extra = []
            if "FETCH_SIZE" in m:
                extra.append("HBM read (FETCH_SIZE x2) = %.1f MB" % (2 * m["FETCH_SIZE"] * 1024 / 1e6))
            if "WRITE_SIZE" in m:
                extra.append("HBM write = %.1f MB" % (m["WRITE_SIZE"] * 1024 / 1e6))
            print("- **%s**: %s" % (kn, ", ".join(extra)))
            for c in sorted(m):
                print("  - %s = %.4g" % (c, m[c]))
        print()


# per-leg profiles (tools/profile_legs.sh: one process per bench leg, 10 launches)
LEG_KERNELS = {
    "c2": ("k_bin", "k_apply", "k_ovf_apply"),
    "exact10": ("k_bin", "k_apply", "k_ovf_apply"),
    "c5": ("k_bin", "k_apply", "k_ovf_apply"),
    "c5_full": ("k_bin", "k_apply", "k_ovf_apply"),
    "c4": ("k_hash_var", "k_bin", "k_apply", "k_ovf_apply"),
    "probe": ("k_probe_sliced",),
    "fset": ("k_fset_sliced",),
    "fset_mixed": ("k_fset_classes",),
    "fset_rows1": ("k_fset_sliced",),
}
LEG_REPS = 10
COUNTERS = {"FETCH_SIZE": "read_bytes", "WRITE_SIZE": "write_bytes", "SQ_INSTS_VALU": "valu_insts",
            "SQ_INSTS_LDS": "lds_insts", "SQ_LDS_IDX_ACTIVE": "lds_idx_active",
            "SQ_LDS_BANK_CONFLICT": "lds_bank_conflict", "SQ_WAVE_CYCLES": "wave_cycles",
            "SQ_BUSY_CYCLES": "busy_cycles", "SQ_WAIT_ANY": "wait_any", "SQ_INSTS_SALU": "salu_insts",
            "GRBM_GUI_ACTIVE": "grbm_gui_active"}


def leg_data(d, leg):
    """Per kernel of the leg: launches per leg iteration, mean duration and
    the mean of every counter per dispatch; and their per-iteration sums."""
    pre = LEG_KERNELS[leg]
    kern = collections.defaultdict(dict)
    ks = os.path.join(d, leg, "stats", "run_kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            kn = short(r["Name"])
            if kn.startswith(pre):
                kern[kn]["calls_per_launch"] = round(int(r["Calls"]) / LEG_REPS, 3)
                kern[kn]["avg_us"] = round(float(r["AverageNs"]) / 1e3, 3)
    for sub in ("fetch", "write", "sq"):
        p = os.path.join(d, leg, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(p)):
            kn = short(r["Kernel_Name"])
            if kn.startswith(pre) and r["Counter_Name"] in COUNTERS:
                vals[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for kn, cv in vals.items():
            for cn, v in cv.items():
                m = sum(v) / len(v)
                if cn == "FETCH_SIZE":
                    m = 2 * m * 1024  # KiB, x2 on gfx950 (MI355X_MICROARCH.md, HBM section)
                elif cn == "WRITE_SIZE":
                    m = m * 1024
                kern[kn][COUNTERS[cn]] = int(m)
    per = collections.Counter()
    for kn, m in kern.items():
        c = m.get("calls_per_launch", 1.0)
        for key in list(COUNTERS.values()) + ["avg_us"]:
            if key in m:
                per[key] += m[key] * c
    out = {k: (round(v, 3) if k == "avg_us" else int(v)) for k, v in per.items()}
    if "avg_us" in out:
        out["kernel_us"] = out.pop("avg_us")
    out["hbm_bytes"] = out.get("read_bytes", 0) + out.get("write_bytes", 0)
    return {"kernels": dict(kern), "per_launch": out}


def legs_json(d, out):
    import json
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    legs = {leg: leg_data(d, leg) for leg in LEG_KERNELS if os.path.isdir(os.path.join(d, leg))}
    json.dump({"profile": os.path.basename(d.rstrip("/")), "format": 2, "kernel_src_sha": bench.build_sources_sha(),
               "legs": legs,
               "note": "per leg iteration (one build / one probe call): sums over its kernels of the mean per "
                       "dispatch x dispatches per iteration; FETCH_SIZE x2 (gfx950), KiB -> B; separate --pmc passes"},
              open(out, "w"), indent=1)
    print("# per-leg rocprofv3 summary: %s\n" % os.path.basename(d.rstrip("/")))
    print("| leg | kernel us | HBM read MB | HBM write MB | VALU inst | LDS inst | LDS-array cycles | GRBM_GUI_ACTIVE |")
    print("|---|---|---|---|---|---|---|---|")
    for leg, v in legs.items():
        p = v["per_launch"]
        print("| %s | %s | %.1f | %.1f | %.4g | %.4g | %.4g | %.4g |" % (
            leg, p.get("kernel_us"), p.get("read_bytes", 0) / 1e6, p.get("write_bytes", 0) / 1e6,
            p.get("valu_insts", 0), p.get("lds_insts", 0), p.get("lds_idx_active", 0), p.get("grbm_gui_active", 0)))
    print()
    for leg, v in legs.items():
        print("## %s\n" % leg)
        for kn, m in v["kernels"].items():
            print("- **%s**: %s" % (kn, ", ".join("%s=%s" % (a, b) for a, b in sorted(m.items()))))
        print()


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[2] == "--json":
        traffic_json(sys.argv[1], sys.argv[3])
    elif len(sys.argv) > 3 and sys.argv[2] == "--legs":
        legs_json(sys.argv[1], sys.argv[3])
    else:
        main(sys.argv[1])
