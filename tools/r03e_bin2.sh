# k_bin2 (specialised hash / flush waves): parity subset, stamps, A/B vs k_bin (LSMB_BIN2=0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03e/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03e/tests.log
[ $rc -le 1 ] || exit $rc
for v in 1 0; do
LSMB_BIN2=$v LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > gpurun_out/r03e/stamp$v.json 2> gpurun_out/r03e/stamp$v.err || exit $?
echo "bin2=$v"; grep stamp gpurun_out/r03e/stamp$v.err | tail -1
done
ab() { LSMB_BIN2=$1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe $2 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "pass_a %.4f pass_b %.4f kernel %.4f step %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], d["ms_per_step"]), d.get("words_equal_oracle_fixture"))' "bin2=$1 $2"; }
for rep in 1 2; do ab 1 ""; ab 0 ""; done
ab 1 "--global-keys 125000000 --filter-keys 1000000000"; ab 0 "--global-keys 125000000 --filter-keys 1000000000"
