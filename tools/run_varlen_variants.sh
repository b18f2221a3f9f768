#!/bin/bash
# C4 var-len build (bench.py's varlen leg; its C2 line runs too, the other legs
# are off) against each variant library: one line per variant with the hash +
# pass A and pass B ms, read from the bench's detail record.
# Usage: tools/run_varlen_variants.sh name1 name2 ...   (name "base" = the product library)
REPO=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $REPO/gpurun_out
for v in "$@"; do
  lib=$REPO/storage-engine_amd/lib/liblsmbloom_$v.so
  [ "$v" = base ] && lib=$REPO/storage-engine_amd/lib/liblsmbloom.so
  det=$REPO/gpurun_out/varlen_$v.json
  LSMB_LIB=$lib timeout -k 10 180 python3 $REPO/bench.py --steps 10 --warmup 3 --no-e2e \
        --no-cpu-baseline --no-probe --no-exact10 --no-c5-full --no-c5 --no-c1 --detail-out $det > /dev/null
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "variant $v failed (rc $rc)"; exit 1; fi
  python3 -c 'import json,sys; d=json.load(open(sys.argv[2]))["varlen"]; print("%-10s hash+pass_a %.4f pass_b %.4f kernel %.4f frac %.3f exact %s" % (sys.argv[1], d["pass_a_ms"], d["pass_b_ms"], d["kernel_ms"], d["frac"], d.get("words_equal_oracle_fixture")))' "$v" "$det"
done
