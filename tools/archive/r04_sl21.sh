#!/bin/bash
# C2 bin width A/B: 2^20-bit bins (913, the product) vs 2^21-bit bins (457:
# half the owners, twice the arrivals per ring, pass B reads each bin twice),
# fresh and accumulate, and two keys per lane where the 2^21 rings hold them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
one() {  # name env... [-- bench args]
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen \
    --no-exact10 --no-probe --no-c1 $EXTRA > /tmp/c2.json 2>/dev/null || return $?
  python3 -c 'import json,sys; a=json.load(open("/tmp/c2.json")); r=a["roofline"]; print("%-22s C2 pass_a %.4f pass_b %.4f kernel %.4f step %.4f exact %s" % (sys.argv[1], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], a["ms_per_step"], a.get("words_equal_oracle_fixture")))' "$name"
}
for rep in 1 2; do
  EXTRA= one fresh_sl20 LSMB_X=0 || exit $?
  EXTRA= one fresh_sl21 LSMB_SLICE_LOG2=21 || exit $?
  EXTRA= one fresh_sl21_wpc2 LSMB_SLICE_LOG2=21 LSMB_BIN_WGS_PER_CU=2 || exit $?
  EXTRA=--accumulate one acc_sl20 LSMB_X=0 || exit $?
  EXTRA=--accumulate one acc_sl21_per1 LSMB_SLICE_LOG2=21 || exit $?
  EXTRA=--accumulate one acc_sl21_per2 LSMB_SLICE_LOG2=21 LSMB_SWEEP_PER=2 || exit $?
done
