#!/bin/bash
# C3 probe at 8 waves per SIMD: k_probe_sliced's C3 instantiation bounded to
# <= 64 VGPRs (liblsmbloom_wpe8.so, -DLSMB_PROBE_WPE=8: 62 VGPRs, no scratch;
# the product has 90) so that two 1024-thread workgroups fit a CU, vs the
# product at one; probe legs, two repetitions, one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04wpe
mkdir -p $OUT
L=$PWD/storage-engine_amd/lib
one() {  # tag lib wgs
  LSMB_LIB=$2 LSMB_PROBE_WGS_PER_CU=$3 timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --no-e2e --no-cpu-baseline \
    --no-varlen --no-exact10 --no-c1 --global-keys 4000000 > $OUT/$1.json 2>$OUT/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); p=d["probe"]; print("%-10s probe %.4f fset %.4f mixed %.4f exact %s %s %s" % (sys.argv[2], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture"), p["fset"].get("answers_equal_oracle_fixture"), p["fset_mixed"].get("answers_equal_oracle_fixture")))' $OUT/$1.json $1
}
for rep in 1 2; do
  one base_w1 $L/liblsmbloom.so 1 || exit $?
  one wpe8_w1 $L/liblsmbloom_wpe8.so 1 || exit $?
  one wpe8_w2 $L/liblsmbloom_wpe8.so 2 || exit $?
done
