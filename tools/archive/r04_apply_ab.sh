#!/bin/bash
# Pass B A/B (k_apply regions per wave round, LSMB_APPLY_SPLIT): C2 and the C5
# shard, product library (base, 1 region per round) vs variants, two repetitions.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/storage-engine_amd/lib
one() {  # name lib
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen \
    --no-exact10 --no-probe --no-c1 > /tmp/c2.json 2>/dev/null || return $?
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 > /tmp/c5.json 2>/dev/null || return $?
  python3 -c 'import json,sys; a=json.load(open("/tmp/c2.json")); b=json.load(open("/tmp/c5.json")); r=a["roofline"]; q=b["roofline"]; print("%-9s C2 pass_a %.4f pass_b %.4f kernel %.4f exact %s | C5 pass_a %.4f pass_b %.4f kernel %.4f" % (sys.argv[1], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], a.get("words_equal_oracle_fixture"), q["pass_a_ms"], q["pass_b_ms"], q["kernel_ms"]))' $1
}
for rep in 1 2; do
  for v in base split2 split4 split2u16; do
    lib=$L/liblsmbloom_$v.so; [ $v = base ] && lib=$L/liblsmbloom.so
    one $v $lib || exit $?
  done
done
