"""bench.py's per-leg roofline objects from a per-leg
PMC summary (profiles/traffic.json format 2): HBM frac from the algorithmic
bytes, traffic from the PMC passes, VALU / LDS busy fractions over the
launch's own cycles, and the stale guard when the kernels' sources change."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _legs(fresh=True):
    return {"source": "profiles/traffic.json (test)", "fresh": fresh, "legs": {"c2": {"per_launch": {
        "hbm_bytes": 6_000_000_000, "read_bytes": 3_500_000_000, "write_bytes": 2_500_000_000,
        "kernel_us": 1500.0, "valu_insts": 400_000_000, "lds_insts": 50_000_000,
        "lds_idx_active": 200_000_000, "lds_bank_conflict": 120_000_000, "grbm_gui_active": 8 * 3_000_000}}}}


def test_leg_roofline_fractions():
    r = bench.leg_roofline("c2", 1_719_589_416, 1.4, "build", legs=_legs())
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - 1_719_589_416 / 1.4e-3 / 1e9 / 8000) < 1e-4
    assert r["traffic"] == 6_000_000_000
    sec = r["secondary"]
    assert sec["launch_cycles"] == 3_000_000
    assert abs(sec["valu"]["frac"] - 400e6 * 4 / (1024 * 3e6)) < 1e-4
    assert abs(sec["lds"]["frac"] - 200e6 / (256 * 3e6)) < 1e-4
    assert abs(sec["lds"]["bank_conflict_share"] - 0.6) < 1e-4
    assert abs(sec["hbm_measured"]["frac"] - 6e9 / 1.5e-3 / 1e9 / 8000) < 1e-4
    busiest = max(("hbm_measured", "valu", "lds"), key=lambda k: sec[k]["frac"])
    assert r["busiest"] == busiest
    # no unit of this launch is near saturation: no limiter is named
    assert sec[busiest]["frac"] < bench.SATURATED and r["limiter"] == "none"


def test_leg_roofline_names_a_saturated_unit():
    legs = _legs()
    legs["legs"]["c2"]["per_launch"]["valu_insts"] = 600_000_000  # 600e6 x 4 / (1024 x 3e6) = 0.78
    r = bench.leg_roofline("c2", 1_719_589_416, 1.4, "build", legs=legs)
    assert r["limiter"] == "valu" and r["secondary"]["valu"]["frac"] >= bench.SATURATED


def test_leg_roofline_stale_and_missing():
    r = bench.leg_roofline("c2", 1e9, 1.0, "build", legs=_legs(fresh=False))
    assert r["traffic"] is None and "traffic_stale" in r and "secondary" not in r
    r = bench.leg_roofline("probe", 1e8, 0.05, "k_probe_sliced", legs=_legs())
    assert r["traffic"] is None and "secondary" not in r and abs(r["frac"] - 1e8 / 0.05e-3 / 1e9 / 8000) < 1e-4


def test_compact_line_fits_the_driver_tail():
    """VERDICT r04 "missing" item 2: the driver keeps ~8 KB of output, so the
    one JSON line must carry every leg (the C3 probe half of the metric
    included) within LINE_BUDGET bytes.  Checked on the committed full record
    of a round-6 run (profiles/r06/r06a_bench_detail.json, every leg present:
    the C5 shard, the 1-GPU C5 point and the one-byte filter-set rows
    included)."""
    import json
    full = json.loads(open(os.path.join(ROOT, "profiles", "r06", "r06a_bench_detail.json")).read())
    full["detail"] = "gpurun_out/bench_detail.json"
    line = json.dumps(bench.compact_line(full), separators=(",", ":"))
    assert len(line) < bench.LINE_BUDGET
    c = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in c, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in c["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c["cpu_baseline"], k
    assert set(c["legs"]) >= {"c3_probe", "fset", "fset_mixed", "fset_rows1", "c2_exact10", "c4", "c5_shard",
                              "c5_full", "c1_gpu", "e2e"}
    assert c["legs"]["c5_shard"]["words_equal_oracle_fixture"] is True
    # the N > 1 curve's same-workload 1-GPU point
    c5f = c["legs"]["c5_full"]
    assert c5f["words_equal_oracle_fixture"] is True and c5f["sweeps"] == 2 and c5f["ms"] > 0
    assert c5f["roofline"]["frac"] > 0 and c5f["value"] > 0
    assert "invalid" not in c and c["value"] > 0
    assert c["legs"]["c3_probe"]["ms"] == full["probe"]["ms"]
    assert c["legs"]["c3_probe"]["answers_equal_oracle_fixture"] is True


def test_invalid_reasons():
    """VERDICT r05 item 1 / ADVICE r05: a line whose own checks fail publishes no
    number — bench.invalid_reasons lists why, main() then sets value null and
    exits non-zero (the GPU test test_bench_fault_nulls_the_value runs it)."""
    assert bench.invalid_reasons({"words_equal_oracle_fixture": True}) == []
    assert bench.invalid_reasons({"words_equal_oracle_fixture": None}) == []  # no fixture for this config
    r = bench.invalid_reasons({"words_equal_oracle_fixture": False, "multi_gpu_merged_equals_single_gpu_build": False})
    assert len(r) == 2
    assert bench.invalid_reasons({"multi_gpu_check_error": "x"}) == ["multi_gpu_check_error"]
    ss = {"step_split": {"flag_timeouts": 2, "merge_poisoned": True}}
    assert bench.invalid_reasons(ss, timed_merge="ipc") and not bench.invalid_reasons(ss, timed_merge="rccl")
    assert bench.invalid_reasons({"step_split": {"flag_timeouts": 0, "merge_poisoned": True}}, timed_merge="ipc")


def test_compact_line_carries_c5_full_and_invalid():
    """the N = 1 line carries legs.c5_full (all 1e9 C5 keys on
    one GPU: the N > 1 curve's same-workload point) within the line budget; an
    invalid line carries its reasons."""
    import json
    full = json.loads(open(os.path.join(ROOT, "profiles", "r05", "r05r_bench_detail.json")).read())
    full["detail"] = "gpurun_out/bench_detail.json"
    full["c5_full"] = {"value": 34000.0, "ms": 29.4, "kernel_ms": 29.4, "sweeps": 2, "words_equal_oracle_fixture": True,
                       "roofline": bench.leg_roofline(None, 16 * 10 ** 9 + 8 * 67108864, 29.4, "build")}
    full["invalid"] = ["words_equal_oracle_fixture is false"]
    line = json.dumps(bench.compact_line(full), separators=(",", ":"))
    assert len(line) < bench.LINE_BUDGET, len(line)
    c = json.loads(line)
    assert c["legs"]["c5_full"]["words_equal_oracle_fixture"] is True and c["legs"]["c5_full"]["sweeps"] == 2
    assert c["legs"]["c5_full"]["roofline"]["frac"] > 0
    assert c["invalid"] == full["invalid"]
