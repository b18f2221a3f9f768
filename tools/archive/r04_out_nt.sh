#!/bin/bash
# Probe / filter-set output rows with the non-temporal policy
# (liblsmbloom_outnt.so, -DLSMB_OUT_NT=1) vs the product: probe legs, two
# repetitions, one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04outnt
mkdir -p $OUT
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --no-e2e --no-cpu-baseline \
    --no-varlen --no-exact10 --no-c1 --global-keys 4000000 > $OUT/$1.json 2>$OUT/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); p=d["probe"]; print("%-8s probe %.4f fset %.4f mixed %.4f exact %s %s %s" % (sys.argv[2], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture"), p["fset"].get("answers_equal_oracle_fixture"), p["fset_mixed"].get("answers_equal_oracle_fixture")))' $OUT/$1.json $1
}
for rep in 1 2 3; do
  one base_$rep $L/liblsmbloom.so || exit $?
  one outnt_$rep $L/liblsmbloom_outnt.so || exit $?
done
