#!/bin/bash
# Ping-pong pass A (k_bin_pp, LSMB_PP=1): the partition-path GPU tests with it
# forced on, then C2 / C4 / exact10 A/B against k_bin (LSMB_PP=0) on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04pp
LSMB_PP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fresh.py tests/test_gpu_random.py \
  tests/test_gpu_block.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04pp/tests.log 2>&1
rc=$?
echo "pp tests rc=$rc"; tail -3 gpurun_out/r04pp/tests.log
[ $rc -eq 0 ] || exit $rc
one() {  # tag pp
  LSMB_PP=$2 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-probe --no-c1 \
    > gpurun_out/r04pp/$1.json 2> gpurun_out/r04pp/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; v=d["varlen"]; x=d["c2_exact_10_bits_per_key"]; print("%-6s C2 step %.4f pass_a %.4f pass_b %.4f kernel %.4f exact %s | C4 pass_a %.4f kernel %.4f exact %s | x10 pass_a %.4f exact %s" % (sys.argv[2], d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], d.get("words_equal_oracle_fixture"), v["pass_a_ms"], v["kernel_ms"], v.get("words_equal_oracle_fixture"), x["pass_a_ms"], x.get("words_equal_oracle_fixture")))' gpurun_out/r04pp/$1.json $1
}
for rep in 1 2; do
  one kbin_$rep 0 || exit $?
  one pp_$rep 1 || exit $?
done
