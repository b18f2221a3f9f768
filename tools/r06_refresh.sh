#!/bin/bash
# Round-6 refresh of the floors DESIGN.md cites (same kernels as round 5):
# the hash + walk floor (tools/mb_hash.hip), the probe's fixed vs per-key cost
# (tools/probe_scale.py), pass A's ablations (LSMB_ABL variants, C2) and the
# LSMB_STAMP phase sections.  Each step under its own time limit; stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
if [ "$2" != "passa" ]; then
timeout -k 10 120 ./tools/mb_hash > $OUT/hash_floor.log 2>&1 || { echo "mb_hash failed"; exit 1; }
cat $OUT/hash_floor.log
timeout -k 10 200 python tools/probe_scale.py > $OUT/probe_scale.jsonl 2> $OUT/probe_scale.err || { echo "probe_scale failed"; exit 1; }
tail -3 $OUT/probe_scale.jsonl
fi
timeout -k 10 600 bash tools/run_variants.sh --no-probe --no-c1 --no-c5 --no-c5-full -- base abl1 abl8 abl16 base abl1 abl8 abl16 > $OUT/ablations.log 2>&1 || { echo "ablations failed"; cat $OUT/ablations.log; exit 1; }
cat $OUT/ablations.log
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 200 python bench.py --steps 10 --warmup 5 --no-probe \
  --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-c1 --no-c5 --no-c5-full > $OUT/stamp_bench.json 2> $OUT/stamps.log
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "stamp run failed"; exit 1; }
grep "\[stamp\]" $OUT/stamps.log | tail -3
