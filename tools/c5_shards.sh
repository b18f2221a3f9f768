#!/bin/bash
# C5 per-GPU shard builds on one GPU: 1e9/N keys into the 2^32-1-bit filter,
# for N = 8, 4, 2 (and optionally 1); prints kernel / pass A / pass B ms.
# Usage: tools/c5_shards.sh [ENV=VAL ...]   (extra env for an A/B variant)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in 125000000 250000000 500000000; do
  env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 2 --global-keys $n --filter-keys 1000000000 \
      --no-probe --no-e2e --no-varlen --no-exact10 --no-cpu-baseline > gpurun_out/c5_$n.json || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/c5_$n.json')); r=d['roofline']
print('$n', '$*', 'step', d['ms_per_step'], 'kernel', r['kernel_ms'], 'A', r['pass_a_ms'], 'B', r['pass_b_ms'], 'Mkeys/s', d['value'])"
done
