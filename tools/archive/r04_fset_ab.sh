#!/bin/bash
# Filter-set kernel A/B (C3 shape, 10 M keys x 8 tables): committed kernel vs
# the rounds kernel with a 64-VGPR cap (product candidate) vs uncapped, at one
# and two 1024-thread workgroups per CU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04s}
mkdir -p gpurun_out/$TAG
L=$PWD/storage-engine_amd/lib
one() {  # tag lib wgs
  LSMB_PROBE_WGS_PER_CU=$3 LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --no-e2e --no-cpu-baseline \
    --no-varlen --no-exact10 --no-c1 --global-keys 4000000 > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); p=d["probe"]; print("%-14s probe %.4f fset %.4f mixed %.4f exact %s %s %s" % (sys.argv[2], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture"), p["fset"].get("answers_equal_oracle_fixture"), p["fset_mixed"].get("answers_equal_oracle_fixture")))' gpurun_out/$TAG/$1.json $1
}
for rep in 1 2; do
  for w in 1 2; do
    [ $w = 1 ] && one prev_w1_$rep $L/liblsmbloom_prev.so 1 || true
    [ $w = 2 ] && one prev_w2_$rep $L/liblsmbloom_prev.so 2 || true
    one cap_w${w}_$rep $L/liblsmbloom.so $w || exit $?
    one nocap_w${w}_$rep $L/liblsmbloom_fsnocap.so $w || exit $?
  done
done
