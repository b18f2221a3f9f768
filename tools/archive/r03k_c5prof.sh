# C5 shard: stamps of pass A's sweep phases, then rocprofv3 kernel stats + PMC passes
cd $GRAFT_REPO_ROOT
O=$PWD/gpurun_out/r03k; mkdir -p $O
C5="--global-keys 125000000 --filter-keys 1000000000 --steps 4 --warmup 1 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10"
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py $C5 > $O/stamp.json 2> $O/stamp.err || exit $?
grep stamp $O/stamp.err | tail -2
timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > /dev/null 2>&1
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe > $O/stamp_c2.json 2> $O/stamp_c2.err || exit $?
grep stamp $O/stamp_c2.err | tail -1
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$O/$name" -o run -- python3 $GRAFT_REPO_ROOT/bench.py $C5 > "$O/$name.log" 2>&1; }
run stats --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run sq1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS || exit $?
run sq2 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES || exit $?
echo done
