# split-VALU pass A: parity subset, stamps, A/B vs the previous pass A
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03d/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03d/tests.log
[ $rc -le 1 ] || exit $rc
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > gpurun_out/r03d/stamp.json 2> gpurun_out/r03d/stamp.err || exit $?
grep stamp gpurun_out/r03d/stamp.err | tail -2
bash tools/run_variants.sh --no-probe -- old base old base
