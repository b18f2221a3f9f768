#!/bin/bash
# (The variant libraries were built from the session tree with tools/build_variants.sh and LSMB_R3_VM /
# LSMB_R3_FLUSH switches that were removed with the experiment; results in profiles/r03/r03_experiments.md.)
# Ablation of the round-3 pass A changes, one box, accumulate builds (zero + lsmb_build_fixed_dev):
# head (6c57a9a) | cur | novm (LSMB_R3_VM=0) | noflush (LSMB_R3_FLUSH=0) | neither; C2 and the C5 shard.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=$PWD/storage-engine_amd/lib
summ='import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("%-18s step %.4f pass_a %.4f pass_b %.4f kernel %.4f" % (sys.argv[1], d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))'
B="--no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-c1 --accumulate"
c2() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 $B | python3 -c "$summ" "$1"; }
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 $B | python3 -c "$summ" "$1"; }
for rep in 1 2; do
  for v in head cur novm noflush neither; do
    if [ $v = cur ]; then L=$D/liblsmbloom.so; else L=$D/liblsmbloom_$v.so; fi
    LSMB_LIB=$L c2 c2_$v || exit $?
    LSMB_LIB=$L c5 c5_$v || exit $?
  done
done
