#!/bin/bash
# A/B of pass A's packed-ring kernel (k_bin_pk, LSMB_PACKED=1) against k_bin
# on the C2 build: GPU parity suite under LSMB_PACKED=1, then bench build legs
# (alternating), then the LSMB_STAMP variant's phase breakdown for both.
# Needs liblsmbloom_st.so (tools/build_variants.sh st="-DLSMB_STAMP=1").
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd $REPO && mkdir -p gpurun_out
LSMB_PACKED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fresh.py tests/test_gpu_random.py tests/test_stream.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05pk_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05pk_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base pk base pk; do
  pk=0; [ $v = pk ] && pk=1
  out=$(LSMB_PACKED=$pk timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline \
        --no-varlen --no-exact10 --no-c1 --no-probe 2>/dev/null) || { echo "bench $v failed"; exit 1; }
  echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("%-5s pass_a %.4f pass_b %.4f kernel %.4f step %.4f exact %s" % (sys.argv[1], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], d["ms_per_step"], d.get("words_equal_oracle_fixture")))' "$v"
done
for pk in 0 1; do
  LSMB_PACKED=$pk LSMB_LIB=$REPO/storage-engine_amd/lib/liblsmbloom_st.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-c1 --no-probe 2>&1 >/dev/null | grep stamp | tail -1 | sed "s/^/packed=$pk /"
done
