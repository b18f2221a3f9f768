#!/bin/bash
# rocprofv3 profile of bench.py on one MI355X (run through gpurun).
# Usage: tools/profile.sh <tag> [extra bench args]
# Writes gpurun_out/prof_<tag>/{stats,fetch,write,sq1,sq2}/; tools/prof_summary.py condenses them.
set -euo pipefail
TAG=${1:-r01}; shift || true
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$REPO/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-varlen --no-exact10 $*"
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 $BENCH > "$OUT/$name.log" 2>&1
}
run stats --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS
run sq2 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES
# C5 shard (125 M keys into the 2^32-1-bit filter: 2 sweeps of 2^21-bit bins),
# kernel trace and HBM bytes (pass B reads each bin's regions for both halves)
C5="$REPO/bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 4 --warmup 1 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_c5" -o run -- python3 $C5 > "$OUT/stats_c5.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_c5" -o run -- python3 $C5 > "$OUT/fetch_c5.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_c5" -o run -- python3 $C5 > "$OUT/write_c5.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/sq1_c5" -o run -- python3 $C5 > "$OUT/sq1_c5.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES \
    --output-format csv -d "$OUT/sq2_c5" -o run -- python3 $C5 > "$OUT/sq2_c5.log" 2>&1
# C4 var-len build kernels (k_bin<ks::VarLen...>, k_apply), kernel trace only
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_c4" -o run -- \
    python3 $REPO/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e --no-probe --no-exact10 --keys-per-gpu 1000000 \
    > "$OUT/stats_c4.log" 2>&1
python3 $REPO/tools/prof_summary.py "$OUT" > "$OUT/summary.md"
python3 $REPO/tools/prof_summary.py "$OUT" --json "$OUT/traffic.json"
echo "profile $TAG done"
