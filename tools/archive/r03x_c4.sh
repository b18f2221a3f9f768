#!/bin/bash
# C4 (100 M var-len keys): head library (6c57a9a) vs this tree (k_hash_var offsets via LDS + coalesced
# record writes), accumulate builds, and this tree's fresh build; one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=$PWD/storage-engine_amd/lib
c4() { local t=$1; shift; timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-exact10 --no-c1 "$@" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline())["varlen"]; print("%-12s pass_a %.4f pass_b %.4f kernel %.4f frac %.4f step %s" % (sys.argv[1], d["pass_a_ms"], d["pass_b_ms"], d["kernel_ms"], d["frac"], d.get("ms_per_step")), d.get("words_equal_oracle_fixture"))' "$t"; }
for rep in 1 2; do
  LSMB_LIB=$D/liblsmbloom_head.so c4 c4_head --accumulate || exit $?
  c4 c4_acc --accumulate || exit $?
  c4 c4_fresh || exit $?
done
