# k_apply with double-buffered region chunks: parity subset, C2 + C5 vs round-2 lib, chunk-size variants
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03l
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "partition or c2 or random or huge or sweep or varlen or c5" > gpurun_out/r03l/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03l/tests.log
[ $rc -le 1 ] || exit $rc
L=$PWD/storage-engine_amd/lib
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "c5 pass_a %.4f pass_b %.4f kernel %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]))' "$1"; }
c2() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "c2 pass_a %.4f pass_b %.4f kernel %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))' "$1"; }
for rep in 1 2; do c5 cur || exit $?; LSMB_LIB=$L/liblsmbloom_r2.so c5 r2 || exit $?; c2 cur || exit $?; LSMB_LIB=$L/liblsmbloom_r2.so c2 r2 || exit $?; done
for v in u4 u6 nt; do LSMB_LIB=$L/liblsmbloom_$v.so c5 $v || exit $?; LSMB_LIB=$L/liblsmbloom_$v.so c2 $v || exit $?; done
LSMB_SWEEP_REC=1 c5 sweeprec || exit $?; LSMB_SWEEP_REC=1 c5 sweeprec || exit $?
