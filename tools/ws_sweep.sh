#!/bin/bash
# C2 build time vs partition workspace limit (key chunking): can a chunk's
# regions + the filter stay Infinity-Cache (MALL) resident?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for mb in 8192 512 256 160 96; do
  LSMB_WORKSPACE_MB=$mb timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-probe --no-e2e --no-varlen \
      --no-exact10 --no-cpu-baseline > gpurun_out/ws_$mb.json || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/ws_$mb.json')); r=d['roofline']
print('ws_mb', $mb, 'step', d['ms_per_step'], 'kernel(last chunk)', r['kernel_ms'], 'A', r['pass_a_ms'], 'B', r['pass_b_ms'])"
done
