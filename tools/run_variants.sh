#!/bin/bash
# GPU side of tools/build_variants.sh: the C2 build (bench.py, build legs only)
# against each variant library; one line per variant with pass A / pass B ms.
# Usage: tools/run_variants.sh [bench args] -- name1 name2 ...   (name "base" = the product library)
REPO=${GRAFT_REPO_ROOT:-/root/repo}
args=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
shift
for v in "$@"; do
  lib=$REPO/storage-engine_amd/lib/liblsmbloom_$v.so
  [ "$v" = base ] && lib=$REPO/storage-engine_amd/lib/liblsmbloom.so
  # (exit 3: the line is invalid because its words fail the oracle check, as
  # an ablation's do by construction; its timings still stand for the A/B)
  out=$(LSMB_LIB=$lib timeout -k 10 120 python3 $REPO/bench.py --steps 20 --warmup 5 --no-e2e \
        --no-cpu-baseline --no-varlen --no-exact10 "${args[@]}")
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "variant $v failed (rc $rc)"; exit 1; fi
  echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; L=d.get("legs", {}); g=lambda n: L.get(n, {}).get("ms"); print("%-10s pass_a %.4f pass_b %.4f kernel %.4f step %.4f exact %s probe %s fset %s mixed %s answers %s" % (sys.argv[1], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], d["ms_per_step"], d.get("words_equal_oracle_fixture"), g("c3_probe"), g("fset"), g("fset_mixed"), [L.get(n, {}).get("answers_equal_oracle_fixture") for n in ("c3_probe", "fset", "fset_mixed")]))' "$v"
done
