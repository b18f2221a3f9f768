#!/bin/bash
# C3 probe A/B on one box: previous probe kernel (lib/liblsmbloom_probe1.so:
# one-deep key prefetch issued after the table build) vs this tree (two-deep,
# first loads before the table build), at one and two 1024-thread workgroups
# per CU (LSMB_PROBE_WGS), two repetitions; probe / fset / fset_mixed ms.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04p
L=$PWD/storage-engine_amd/lib
one() {  # tag lib wgs
  LSMB_PROBE_WGS_PER_CU=$3 LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --no-e2e --no-cpu-baseline \
    --no-varlen --no-exact10 --no-c1 --global-keys 4000000 > gpurun_out/r04p/$1.json 2> gpurun_out/r04p/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); p=d["probe"]; print("%-10s probe %.4f fset %.4f mixed %.4f exact %s %s %s" % (sys.argv[2], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture"), p["fset"].get("answers_equal_oracle_fixture"), p["fset_mixed"].get("answers_equal_oracle_fixture")))' gpurun_out/r04p/$1.json $1
}
for rep in 1 2; do
  for w in 1 2; do
    one prev_w${w}_$rep $L/liblsmbloom_probe1.so $w || exit $?
    one cur_w${w}_$rep $L/liblsmbloom.so $w || exit $?
  done
done
