#!/bin/bash
# C5 shard A/B on one box (125 M keys into new(1e9, 0.01) = 2^32-1 bits, fresh
# sweeps): lib/liblsmbloom_prev.so (the committed kernels) vs
# this tree (r04m: WalkM; r04ab: branch-free half select in k_apply<21>), two reps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04m}
mkdir -p gpurun_out/$TAG
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 5 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print("%-8s C5 step %.4f kernel %.4f pass_a %.4f pass_b %.4f" % (sys.argv[2], d["ms_per_step"], r["kernel_ms"], r["pass_a_ms"], r["pass_b_ms"]))' gpurun_out/$TAG/$1.json $1
}
for rep in 1 2; do
  one prev_$rep $L/liblsmbloom_prev.so || exit $?
  one cur_$rep $L/liblsmbloom.so || exit $?
done
