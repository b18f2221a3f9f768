#!/bin/bash
# A/B of pass A's flush with every round's job and ring reads hoisted ahead
# of the stores (product source) against the committed one-round-at-a-time
# flush (liblsmbloom_old.so), then the LSMB_STAMP=2 flush split of the new one.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fresh.py tests/test_gpu_random.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r05v_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05v_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/run_variants.sh --no-c1 --no-probe --no-c5 -- old base old base || exit 1
for v in st2; do
  LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_$v.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e \
    --no-cpu-baseline --no-varlen --no-exact10 --no-c1 --no-probe --no-c5 2>&1 >/dev/null | grep stamp | tail -2 | sed "s/^/$v /"
done
