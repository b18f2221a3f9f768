#!/bin/bash
# Fresh-build entry points (lsmb_build_*_dev_new): their GPU tests + the
# partition parity subset, then the C2 bench line and the C5 shard timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fresh.py tests/test_gpu_parity.py -m gpu --maxfail=3 -v --timeout 300 --timeout-method thread -k "fresh or multi_sweep or duplicate or huge or fixed16 or or_acc or c4_10m or tiled or any_k" > gpurun_out/r03s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03s_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03s_bench.json 2> gpurun_out/r03s_bench.err || exit $?
python3 -c 'import json; d=json.load(open("gpurun_out/r03s_bench.json")); r=d["roofline"]; print("c2", d["value"], d["ms_per_step"], r["kernel_ms"], r["pass_a_ms"], r["pass_b_ms"], d.get("words_equal_oracle_fixture"))'
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("c5 step %.4f pass_a %.4f pass_b %.4f kernel %.4f" % (d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))'; }
c5
