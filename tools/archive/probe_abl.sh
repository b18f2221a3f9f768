#!/bin/bash
# C3 probe ablations: product, no table reads, no XXH3, no position walk.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in product pabl1 pabl2 pabl3; do
  lib=storage-engine_amd/lib/liblsmbloom.so; [ $v != product ] && lib=storage-engine_amd/lib/liblsmbloom_$v.so
  LSMB_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-e2e --no-varlen --no-exact10 \
      --no-cpu-baseline --global-keys 1000000 > gpurun_out/pa_$v.json || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/pa_$v.json'))['probe']; print('$v', d['ms'])"
done
