#!/bin/bash
# WRITE_SIZE calibration for scattered 64-B segment writes (tools/mb_wsize.hip).
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/wsize
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $REPO/storage-engine_amd/build/mb_wsize > "$OUT/time.log" 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $REPO/storage-engine_amd/build/mb_wsize > "$OUT/write.log" 2>&1
cat "$OUT/time.log"
python3 - "$OUT/write/run_counter_collection.csv" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "WRITE_SIZE":
        v[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))  # (no namespaces here)
for k, x in v.items():
    gb = sum(x) / len(x) * 1024 / 1e9
    print("%-40s WRITE_SIZE %.3f GB per launch = %.3f x the 2.147 GB written" % (k[:40], gb, gb / 2.147483648))
PY
