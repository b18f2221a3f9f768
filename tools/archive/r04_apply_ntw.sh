#!/bin/bash
# Pass B slice write-back with the non-temporal policy (liblsmbloom_ntw.so,
# -DLSMB_APPLY_NTW=1) vs the product: C2 + C5 shard, two repetitions, one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/r04ntw
mkdir -p $OUT
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 180 python3 bench.py --steps 20 --warmup 10 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 \
    --no-probe --no-c1 > $OUT/$1.json 2> $OUT/$1.err || return $?
  LSMB_LIB=$2 timeout -k 10 180 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 5 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 > $OUT/$1_c5.json 2>> $OUT/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); e=json.load(open(sys.argv[2])); r=d["roofline"]; q=e["roofline"]; print("%-7s C2 kernel %.4f pass_a %.4f pass_b %.4f exact %s | C5 kernel %.4f pass_a %.4f pass_b %.4f" % (sys.argv[3], r["kernel_ms"], r["pass_a_ms"], r["pass_b_ms"], d.get("words_equal_oracle_fixture"), q["kernel_ms"], q["pass_a_ms"], q["pass_b_ms"]))' $OUT/$1.json $OUT/$1_c5.json $1
}
for rep in 1 2; do
  one base_$rep $L/liblsmbloom.so || exit $?
  one ntw_$rep $L/liblsmbloom_ntw.so || exit $?
done
