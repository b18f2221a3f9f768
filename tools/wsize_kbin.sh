#!/bin/bash
# WRITE_SIZE of k_bin (C2) for the product and two ablations: every region
# store dropped (LSMB_ABL=16) and no flush at all (LSMB_ABL=1).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/wsize_kbin
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in product abl16 abl1; do
  lib=$REPO/storage-engine_amd/lib/liblsmbloom.so
  [ $v != product ] && lib=$REPO/storage-engine_amd/lib/liblsmbloom_$v.so
  LSMB_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$v" -o run -- \
    python3 $REPO/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-probe \
    > "$OUT/$v.log" 2>&1 || exit $?
  python3 - "$OUT/$v/run_counter_collection.csv" $v <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "WRITE_SIZE":
        v[r["Kernel_Name"].replace("lsmb::(anonymous namespace)::", "")].append(float(r["Counter_Value"]))
for k, x in v.items():
    if "k_bin" in k or "k_apply" in k or "Fill" in k:
        print(sys.argv[2], "%-60s WRITE_SIZE %.3f GB per launch (n=%d)" % (k[-60:], sum(x) / len(x) * 1024 / 1e9, len(x)))
PY
done
