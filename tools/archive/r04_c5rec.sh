#!/bin/bash
# rocprofv3 kernel stats of tools/r04_c5rec.py (C5 shard: fixed-16 sweeps vs
# sweeps replaying k_hash_var's walk records).
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r04c5rec
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
  -- python3 $REPO/tools/r04_c5rec.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
grep "filters equal" $OUT/run.log
python3 - $OUT <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/prof/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Name"].startswith(("void lsmb", "lsmb")):
            print("%-90s calls %4s avg_us %9.1f" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
