#!/bin/bash
# Pass A timing ablations (tools only): runs bench.py's C2 build against the
# LSMB_ABL-instrumented libraries built by tools/build_abl.sh.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
for v in 0 "$@"; do
  lib=$REPO/storage-engine_amd/lib/liblsmbloom_abl$v.so
  [ "$v" = 0 ] && lib=$REPO/storage-engine_amd/lib/liblsmbloom.so
  echo "== abl $v"
  LSMB_LIB=$lib timeout -k 10 120 python3 $REPO/bench.py --steps 10 --warmup 3 --no-probe --no-e2e --no-cpu-baseline \
    | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("pass_a %.4f pass_b %.4f step %.4f" % (r["pass_a_ms"], r["pass_b_ms"], d["ms_per_step"]))' || exit 1
done
