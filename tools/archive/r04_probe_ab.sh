#!/bin/bash
# C3 probe A/B on one box: the committed kernel (lib/liblsmbloom_prev.so) vs
# this tree, two repetitions each; probe / fset / fset_mixed ms and the
# full-size answer digests.  r04p: one- vs two-deep prefetch (dropped);
# r04q: grid-wide rounds through scalar-advanced buffer resources, three
# rounds in flight, first keys requested before the table build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04q}
mkdir -p gpurun_out/$TAG
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --no-e2e --no-cpu-baseline \
    --no-varlen --no-exact10 --no-c1 --global-keys 4000000 > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); p=d["probe"]; print("%-10s probe %.4f fset %.4f mixed %.4f exact %s %s %s" % (sys.argv[2], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture"), p["fset"].get("answers_equal_oracle_fixture"), p["fset_mixed"].get("answers_equal_oracle_fixture")))' gpurun_out/$TAG/$1.json $1
}
for rep in 1 2; do
  one prev_$rep $L/liblsmbloom_prev.so || exit $?
  one cur_$rep $L/liblsmbloom.so || exit $?
done
