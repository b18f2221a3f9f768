#!/bin/bash
# Bin width A/B where 2^20-bit bins need exactly 2 sweeps: C2 exact 10 bits/key
# (1e9 bits) and a new(2e8, .01) filter (1.9e9 bits), 100 M keys each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for env in LSMB_SLICE_LOG2=20 LSMB_SLICE_LOG2=21; do
  env $env timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-probe --no-e2e --no-varlen --no-cpu-baseline \
      > gpurun_out/sl_ab_a.json || exit $?
  env $env timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-probe --no-e2e --no-varlen --no-cpu-baseline \
      --no-exact10 --filter-keys 200000000 > gpurun_out/sl_ab_b.json || exit $?
  python3 -c "
import json; a=json.load(open('gpurun_out/sl_ab_a.json')); b=json.load(open('gpurun_out/sl_ab_b.json'))
e=a['c2_exact_10_bits_per_key']; r=b['roofline']
print('$env', 'exact10 kernel', e['kernel_ms'], 'A', e['pass_a_ms'], 'B', e['pass_b_ms'], '| 2e8 filter kernel', r['kernel_ms'], 'A', r['pass_a_ms'], 'B', r['pass_b_ms'])"
done
