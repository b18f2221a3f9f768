#!/bin/bash
# Pass A workgroups per CU (LSMB_BIN_WGS_PER_CU): C2 and the C5 N=8 shard.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 1 2 3; do
  LSMB_BIN_WGS_PER_CU=$w timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-probe --no-e2e --no-varlen \
      --no-exact10 --no-cpu-baseline > gpurun_out/bw_c2_$w.json || exit $?
  LSMB_BIN_WGS_PER_CU=$w timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-probe --no-e2e --no-varlen \
      --no-exact10 --no-cpu-baseline --global-keys 125000000 --filter-keys 1000000000 > gpurun_out/bw_c5_$w.json || exit $?
  python3 -c "
import json; a=json.load(open('gpurun_out/bw_c2_$w.json'))['roofline']; b=json.load(open('gpurun_out/bw_c5_$w.json'))['roofline']
print('wgs/cu $w C2', a['kernel_ms'], a['pass_a_ms'], a['pass_b_ms'], '| C5 shard', b['kernel_ms'], b['pass_a_ms'], b['pass_b_ms'])"
done
