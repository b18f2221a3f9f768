#!/bin/bash
# C3 probe / filter set vs 1024-thread workgroups per CU (LSMB_PROBE_WGS_PER_CU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 1 2 3 4; do
  LSMB_PROBE_WGS_PER_CU=$w timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-e2e --no-varlen --no-exact10 \
      --no-cpu-baseline --global-keys 1000000 > gpurun_out/pw_$w.json || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/pw_$w.json'))['probe']; print('wgs/cu $w probe', d['ms'], 'fset', d['fset']['ms'], 'mixed', d['fset_mixed']['ms'])"
done
