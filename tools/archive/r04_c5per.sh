#!/bin/bash
# C5 shard with the fold walk: fresh sweeps (one key per lane, overflow lists)
# vs accumulate with two keys per lane (the plan's default there; overflow to
# the words by global atomics) vs accumulate forced to one key per lane.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04cp
one() {  # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 5 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 $EXTRA > gpurun_out/r04cp/$tag.json 2>/dev/null || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print("%-12s C5 step %.4f kernel %.4f pass_a %.4f pass_b %.4f" % (sys.argv[2], d["ms_per_step"], r["kernel_ms"], r["pass_a_ms"], r["pass_b_ms"]))' gpurun_out/r04cp/$tag.json $tag
}
for rep in 1 2; do
  EXTRA= one fresh_per1 LSMB_X=0 || exit $?
  EXTRA=--accumulate one acc_per2 LSMB_X=0 || exit $?
  EXTRA=--accumulate one acc_per1 LSMB_SWEEP_PER=1 || exit $?
done
