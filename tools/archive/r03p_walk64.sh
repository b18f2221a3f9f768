# Walk64 / RecWalk64 as 32-bit adds with carry-out (no 64-bit sums): full GPU suite, then C5 + C2 vs round-2 lib
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03p
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=3 -q --timeout 300 --timeout-method thread > gpurun_out/r03p/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03p/tests.log
[ $rc -le 1 ] || exit $rc
R2=$PWD/storage-engine_amd/lib/liblsmbloom_r2.so
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "c5 pass_a %.4f pass_b %.4f kernel %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]))' "$1"; }
for rep in 1 2; do c5 cur || exit $?; LSMB_LIB=$R2 c5 r2 || exit $?; done
