#!/bin/bash
# C4 var-len build (bench.py's varlen leg only) against each variant library:
# one line per variant with the hash + pass A and pass B ms.
# Usage: tools/run_varlen_variants.sh name1 name2 ...   (name "base" = the product library)
REPO=${GRAFT_REPO_ROOT:-/root/repo}
for v in "$@"; do
  lib=$REPO/storage-engine_amd/lib/liblsmbloom_$v.so
  [ "$v" = base ] && lib=$REPO/storage-engine_amd/lib/liblsmbloom.so
  out=$(LSMB_LIB=$lib timeout -k 10 180 python3 $REPO/bench.py --steps 10 --warmup 3 --no-e2e \
        --no-cpu-baseline --no-probe --no-exact10) || { echo "variant $v failed"; exit 1; }
  echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline())["varlen"]; print("%-10s hash+pass_a %.4f pass_b %.4f kernel %.4f frac %.3f exact %s" % (sys.argv[1], d["pass_a_ms"], d["pass_b_ms"], d["kernel_ms"], d["frac"], d.get("words_equal_oracle_fixture")))' "$v"
done
