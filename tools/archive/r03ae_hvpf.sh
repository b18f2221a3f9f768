#!/bin/bash
# C4 k_hash_var: HEAD (one workgroup per block; lib/liblsmbloom_head.so) vs a
# grid of 4 workgroups per CU that each hash a run of blocks with the next
# block's bounds prefetched by LDS-DMA (the product), two repetitions.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  bash tools/run_varlen_variants.sh head base || exit $?
done
