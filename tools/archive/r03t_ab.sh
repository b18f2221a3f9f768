#!/bin/bash
# A/B on one box: HEAD library (liblsmbloom_head.so, 6c57a9a) vs this tree, C2 and the C5 shard;
# --accumulate = zero + the OR-accumulate build, else the fresh build (lsmb_build_fixed_dev_new).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
H=$PWD/storage-engine_amd/lib/liblsmbloom_head.so
summ='import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("%-22s step %.4f pass_a %.4f pass_b %.4f kernel %.4f" % (sys.argv[1], d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))'
c2() { local tag=$1; shift; timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-c1 "$@" | python3 -c "$summ" "$tag"; }
c5() { local tag=$1; shift; timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-c1 "$@" | python3 -c "$summ" "$tag"; }
for rep in 1 2; do
  LSMB_LIB=$H c2 c2_head_acc --accumulate || exit $?
  c2 c2_new_acc --accumulate || exit $?
  c2 c2_new_fresh || exit $?
done
for rep in 1 2; do
  LSMB_LIB=$H c5 c5_head_acc --accumulate || exit $?
  c5 c5_new_acc --accumulate || exit $?
  c5 c5_new_fresh_per1 || exit $?
  LSMB_SWEEP_PER=1 LSMB_LIB=$H c5 c5_head_acc_per1 --accumulate || exit $?
done
