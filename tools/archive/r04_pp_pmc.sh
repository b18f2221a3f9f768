#!/bin/bash
# Why the ping-pong pass A loses (tools/archive/r04_pingpong_passA.patch):
# SQ activity of k_bin (LSMB_PP=0) and k_bin_pp (LSMB_PP=1, lib
# liblsmbloom_pp.so) on the C2 leg.  SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* /
# SQ_WAIT_* count quad-cycles per wave, summed over waves.
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r04ppmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for pp in 0 1; do
  LSMB_PP=$pp LSMB_LIB=$REPO/storage-engine_amd/lib/liblsmbloom_pp.so timeout -k 10 240 rocprofv3 \
    --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES \
    --output-format csv -d $OUT/pp$pp -o run -- python3 $REPO/tools/legs.py c2 --reps 5 > $OUT/pp$pp.log 2>&1 || exit $?
  python3 - $OUT/pp$pp/run_counter_collection.csv $pp <<'PY'
import csv, collections, sys
v = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if r["Kernel_Name"].split("(")[0].split("::")[-1].startswith("k_bin"):
        v[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in v.items():
    m = {c: sum(x) / len(x) for c, x in cs.items()}
    wc = m["SQ_WAVE_CYCLES"]
    print("LSMB_PP=%s %s: wave-cycles %.4g, VALU active %.3f, LDS active %.3f, LDS wait %.3f, any wait %.3f of wave cycles; VALU insts %.4g, LDS insts %.4g"
          % (sys.argv[2], k[:40], wc, m["SQ_ACTIVE_INST_VALU"] / wc, m["SQ_ACTIVE_INST_LDS"] / wc, m["SQ_WAIT_INST_LDS"] / wc,
             m["SQ_WAIT_ANY"] / wc, m["SQ_INSTS_VALU"], m["SQ_INSTS_LDS"]))
PY
done
