#!/bin/bash
# k_hash_var block bounds from an XCD-ordered table (k_hv_bounds; an L2 hit
# for 7 blocks of 8) vs from the offsets (an HBM round trip before each
# block's first window load, LSMB_HV_NO_BOUNDS=1), same library, one box:
# the var-len GPU tests, the C4 bench leg twice each way, then rocprofv3
# kernel stats of the C4 leg each way.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04hvb}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block.py tests/test_gpu_fresh.py -m gpu -x -q \
  -k "var or c4 or 4gib or block" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
one() {  # tag no_bounds
  env ${2:+LSMB_HV_NO_BOUNDS=1} timeout -k 10 180 python3 bench.py --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-exact10 \
    --no-c1 --no-probe > $OUT/$1.json 2> $OUT/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); v=d["varlen"]; print("%-8s C4 kernel %.4f pass_a %.4f pass_b %.4f exact %s" % (sys.argv[2], v["kernel_ms"], v["pass_a_ms"], v["pass_b_ms"], v.get("words_equal_oracle_fixture")))' $OUT/$1.json $1
}
for rep in 1 2; do
  one offs_$rep 1 || exit $?
  one table_$rep "" || exit $?
done
cd /tmp && export TMPDIR=/tmp
for v in offs table; do
  nb=""; [ $v = offs ] && nb=1
  LSMB_HV_NO_BOUNDS=$nb timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/legs.py c4 --reps 5 > $OUT/prof_$v.log 2>&1 || exit $?
done
python3 - $OUT <<'PY'
import csv, glob, sys
for v in ("offs", "table"):
    for f in glob.glob(sys.argv[1] + "/prof_%s/**/run_kernel_stats.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Name"].startswith(("k_hash_var", "k_hv_bounds", "k_bin", "k_apply")):
                print("%-6s %-60s calls %5s avg_us %9.1f" % (v, r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
