# default bench line (C2 + C4 records + C3) and the C5 shard, current product
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err || exit $?
timeout -k 10 300 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 > gpurun_out/r03h/c5.json 2> gpurun_out/r03h/c5.err || exit $?
python3 - <<'P'
import json
for f in ("bench", "c5"):
    d = json.loads(open("gpurun_out/r03h/%s.json" % f).readline())
    r = d["roofline"]
    print(f, "ms", d["ms_per_step"], "frac", r["frac"], "pa", r.get("pass_a_ms"), "pb", r.get("pass_b_ms"), "kern", r.get("kernel_ms"), d.get("words_equal_oracle_fixture"))
    for k, v in d.items():
        if isinstance(v, dict) and k not in ("roofline", "config", "cpu_baseline"): print(" ", k, json.dumps(v)[:400])
P
