#!/bin/bash
# C4 A/B on one box, the varlen bench leg (100 M C4 keys, fresh build), two
# repetitions: lib/liblsmbloom_prev.so (LdsReader loads built from aligned
# dwords with v_alignbit), r31 (byte-aligned ds_reads + 32-bit remainders in
# the walk records), this tree (+ the 129-240 B extra rounds unrolled).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04y}
mkdir -p gpurun_out/$TAG
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 180 python3 bench.py --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-exact10 \
    --no-c1 --no-probe > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); v=d["varlen"]; print("%-8s C4 kernel %.4f pass_a %.4f pass_b %.4f exact %s | C2 kernel %.4f" % (sys.argv[2], v["kernel_ms"], v["pass_a_ms"], v["pass_b_ms"], v.get("words_equal_oracle_fixture"), d["roofline"]["kernel_ms"]))' gpurun_out/$TAG/$1.json $1
}
for rep in 1 2; do
  one prev_$rep $L/liblsmbloom_prev.so || exit $?
  [ -f $L/liblsmbloom_r31.so ] && { one r31_$rep $L/liblsmbloom_r31.so || exit $?; }
  one cur_$rep $L/liblsmbloom.so || exit $?
done
