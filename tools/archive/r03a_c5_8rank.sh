set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
( while sleep 30; do echo tick $(date +%T); done ) &
TICK=$!
timeout -k 10 600 python3 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 > gpurun_out/r03a/c5_8rank.json 2> gpurun_out/r03a/c5_8rank.err
rc=$?
echo "8rank rc=$rc"
cd /tmp && export TMPDIR=/tmp
[ $rc -eq 0 ] && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03a/c5shard -o run -- python3 $GRAFT_REPO_ROOT/bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 > $GRAFT_REPO_ROOT/gpurun_out/r03a/c5shard.json 2>&1
rc2=$?
kill $TICK
echo "c5shard rc=$rc2"
exit $rc
