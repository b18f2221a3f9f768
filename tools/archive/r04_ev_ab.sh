#!/bin/bash
# Event-marker A/B on one box: lib/liblsmbloom_prev.so (guard events recorded
# with hipEventRecord after each build / probe) vs this tree (completed by the
# last kernel's own dispatch, hipExtLaunchKernelGGL), C2 step + C5 shard step
# + probe legs, two repetitions.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04x}
mkdir -p gpurun_out/$TAG
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen \
    --no-exact10 --no-c1 > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || return $?
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 > gpurun_out/$TAG/$1_c5.json 2>> gpurun_out/$TAG/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); e=json.load(open(sys.argv[2])); r=d["roofline"]; p=d["probe"]; print("%-8s C2 step %.4f kernel %.4f exact %s | C5 step %.4f kernel %.4f | probe %.4f fset %.4f mixed %.4f exact %s" % (sys.argv[3], d["ms_per_step"], r["kernel_ms"], d.get("words_equal_oracle_fixture"), e["ms_per_step"], e["roofline"]["kernel_ms"], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture")))' gpurun_out/$TAG/$1.json gpurun_out/$TAG/$1_c5.json $1
}
for rep in 1 2; do
  one prev_$rep $L/liblsmbloom_prev.so || exit $?
  one cur_$rep $L/liblsmbloom.so || exit $?
done
