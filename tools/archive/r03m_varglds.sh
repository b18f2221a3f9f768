# k_hash_var with the first window issued as LDS-DMA before the lane sort: parity (var-len tests) + C4 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03m
L=$PWD/storage-engine_amd/lib
LSMB_LIB=$L/liblsmbloom_glds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block.py -m gpu -x -q --timeout 200 --timeout-method thread -k "var or c4 or block" > gpurun_out/r03m/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03m/tests.log
[ $rc -le 1 ] || exit $rc
c4() { timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline())["varlen"]; print(sys.argv[1], "pass_a %.4f pass_b %.4f kernel %.4f frac %.4f" % (d["pass_a_ms"], d["pass_b_ms"], d["kernel_ms"], d["frac"]), d.get("words_equal_oracle_fixture"))' "$1"; }
for rep in 1 2; do c4 cur || exit $?; LSMB_LIB=$L/liblsmbloom_glds.so c4 glds || exit $?; done
