#!/bin/bash
# Probe legs at one and two 1024-thread workgroups per CU (LSMB_PROBE_WGS_PER_CU)
# with the round-4 kernels (rounds, transposed tables), two repetitions.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04pw
for rep in 1 2; do
  for w in 1 2 3; do
    LSMB_PROBE_WGS_PER_CU=$w timeout -k 10 120 python3 bench.py --steps 50 --warmup 5 --no-e2e --no-cpu-baseline \
      --no-varlen --no-exact10 --no-c1 --global-keys 4000000 > gpurun_out/r04pw/w$w.json 2>/dev/null || exit $?
    python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); p=d["probe"]; print("wgs %s probe %.4f fset %.4f mixed %.4f exact %s %s %s" % (sys.argv[2], p["ms"], p["fset"]["ms"], p["fset_mixed"]["ms"], p.get("answers_equal_oracle_fixture"), p["fset"].get("answers_equal_oracle_fixture"), p["fset_mixed"].get("answers_equal_oracle_fixture")))' gpurun_out/r04pw/w$w.json $w
  done
done
