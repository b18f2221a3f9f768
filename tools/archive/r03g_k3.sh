# k_bin three-section phase (LSMB_K3): parity on the variant, stamps, A/B vs base (C2)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03g
K3=$PWD/storage-engine_amd/lib/liblsmbloom_k3.so
LSMB_LIB=$K3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "partition or c2 or random or huge or sweep" > gpurun_out/r03g/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03g/tests.log
[ $rc -le 1 ] || exit $rc
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_k3stamp.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > gpurun_out/r03g/stamp.json 2> gpurun_out/r03g/stamp.err || exit $?
grep stamp gpurun_out/r03g/stamp.err | tail -1
ab() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "pass_a %.4f pass_b %.4f kernel %.4f step %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"], d["ms_per_step"]), d.get("words_equal_oracle_fixture"))' "$1"; }
for rep in 1 2; do LSMB_LIB=$K3 ab k3 || exit $?; ab base || exit $?; done
