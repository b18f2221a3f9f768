# pass A phase-section stamps (diagnostic build) + base / no-flush A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03c
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > gpurun_out/r03c/stamp.json 2> gpurun_out/r03c/stamp.err || exit $?
grep stamp gpurun_out/r03c/stamp.err | tail -3
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > gpurun_out/r03c/stamp5.json 2> gpurun_out/r03c/stamp5.err || exit $?
grep stamp gpurun_out/r03c/stamp5.err | tail -2
bash tools/run_variants.sh --no-probe -- base abl1 base abl1
