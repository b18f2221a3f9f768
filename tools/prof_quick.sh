#!/bin/bash
# Quick rocprofv3 passes over the C2 build legs of bench.py (kernel stats, HBM
# fetch / write, L2 hit / miss, SQ mix) -> gpurun_out/ps_<tag>/
TAG=${1:-x}; shift || true
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/pq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$REPO/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-probe $*"
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 $BENCH > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }
}
run stats --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run l2 --pmc TCC_HIT_sum TCC_MISS_sum
run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT
python3 $REPO/tools/prof_summary.py "$OUT" > "$OUT/summary.md"
echo "profile $TAG done"
