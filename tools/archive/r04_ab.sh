#!/bin/bash
# A/B on one box: round-3 library (lib/liblsmbloom_r3.so, built from 3dcef81)
# vs this tree, C2 build + C3 probe legs, two repetitions each, then pass A's
# phase-section stamps (LSMB_STAMP builds) of both.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04ab
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen \
    --no-exact10 --no-c1 > gpurun_out/r04ab/$1.json 2> gpurun_out/r04ab/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; p=d["probe"]; print("%-8s step %.4f pass_a %.4f pass_b %.4f kernel %.4f probe %.4f fset %.4f exact %s %s" % (sys.argv[2], d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], p["ms"], p["fset"]["ms"], d.get("words_equal_oracle_fixture"), p.get("answers_equal_oracle_fixture")))' gpurun_out/r04ab/$1.json $1
}
for rep in 1 2; do
  one r3_$rep $L/liblsmbloom_r3.so || exit $?
  one cur_$rep $L/liblsmbloom.so || exit $?
done
for v in r3stamp stamp; do
  LSMB_LIB=$L/liblsmbloom_$v.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline \
    --no-varlen --no-exact10 --no-probe --no-c1 > gpurun_out/r04ab/$v.json 2> gpurun_out/r04ab/$v.err || exit $?
  echo "$v: $(grep stamp gpurun_out/r04ab/$v.err | tail -1)"
done
