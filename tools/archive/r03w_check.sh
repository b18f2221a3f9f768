#!/bin/bash
# fresh-build + partition parity subset, then head vs this tree (accumulate and fresh), C2 and the C5 shard
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fresh.py tests/test_gpu_parity.py tests/test_gpu_random.py -m gpu --maxfail=3 -q --timeout 300 --timeout-method thread -k "fresh or multi_sweep or duplicate or huge or or_acc or any_k or c4_10m or random or fixed16 or tiled or device_api" > gpurun_out/r03w_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03w_tests.log; [ $rc -ne 0 ] && exit $rc
D=$PWD/storage-engine_amd/lib
summ='import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("%-18s step %.4f pass_a %.4f pass_b %.4f kernel %.4f" % (sys.argv[1], d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))'
B="--no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-c1"
c2() { local t=$1; shift; timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 $B "$@" | python3 -c "$summ" "$t"; }
c5() { local t=$1; shift; timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 $B "$@" | python3 -c "$summ" "$t"; }
for rep in 1 2; do
  LSMB_LIB=$D/liblsmbloom_head.so c2 c2_head_acc --accumulate || exit $?
  c2 c2_acc --accumulate || exit $?
  c2 c2_fresh || exit $?
  LSMB_LIB=$D/liblsmbloom_head.so c5 c5_head_acc --accumulate || exit $?
  c5 c5_acc --accumulate || exit $?
  c5 c5_fresh || exit $?
done
