#!/bin/bash
# Multi-sweep fixed-16 builds: sweep 0 writes every key's (h1, h2) with
# non-temporal stores (liblsmbloom_nt.so) or its 12-B walk record
# (liblsmbloom_rec12.so), later sweeps walk from them, vs every sweep
# hashing the keys (LSMB_NO_EMIT=1), one
# box: the sweep / C5 GPU tests, the C5 shard bench leg twice each way,
# rocprofv3 kernel stats of the C5 leg each way.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04emit}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fresh.py tests/test_gpu_block.py -m gpu -x -q \
  -k "sweep or c5 or saturat or multichunk or fresh" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/storage-engine_amd/lib
one() {  # tag no_emit [lib]
  LSMB_LIB=${3:-$L/liblsmbloom.so} LSMB_NO_EMIT=$2 timeout -k 10 180 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 5 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 > $OUT/$1.json 2> $OUT/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print("%-8s C5 shard step %.4f kernel %.4f pass_a %.4f pass_b %.4f" % (sys.argv[2], d["ms_per_step"], r["kernel_ms"], r["pass_a_ms"], r["pass_b_ms"]))' $OUT/$1.json $1
}
for rep in 1 2; do
  one hash_$rep 1 || exit $?
  one nt_$rep 0 $L/liblsmbloom_nt.so || exit $?
  one rec12_$rep 0 $L/liblsmbloom_rec12.so || exit $?
done
cd /tmp && export TMPDIR=/tmp
for v in hash nt rec12; do
  ne=0; [ $v = hash ] && ne=1
  lib=$L/liblsmbloom.so; [ $v != hash ] && lib=$L/liblsmbloom_$v.so
  LSMB_LIB=$lib LSMB_NO_EMIT=$ne timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/legs.py c5 --reps 5 > $OUT/prof_$v.log 2>&1 || exit $?
done
python3 - $OUT <<'PY'
import csv, glob, sys
for v in ("hash", "nt", "rec12"):
    for f in glob.glob(sys.argv[1] + "/prof_%s/**/run_kernel_stats.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Name"].startswith(("void lsmb", "lsmb")) and "gen_" not in r["Name"]:
                print("%-5s %-80s calls %4s avg_us %8.1f" % (v, r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
