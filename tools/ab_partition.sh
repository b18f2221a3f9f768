#!/bin/bash
# A/B of the partition pass A: sorted tiles (default) vs rings, plus the GPU parity suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "parity or block or multi" > gpurun_out/$1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$1_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in ${VARIANTS:-sortr flat ring}; do
  LSMB_PARTITION=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 > gpurun_out/$1_$v.json 2> gpurun_out/$1_$v.err || exit $?
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); r=d["roofline"]; print(sys.argv[2], "pass_a %.4f pass_b %.4f kernel %.4f step %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], d["ms_per_step"]), d.get("words_equal_oracle_fixture"))' gpurun_out/$1_$v.json $v
done
