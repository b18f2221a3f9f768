#!/bin/bash
# A/B of C5 shard builds: 2^20 bins (4 sweeps) vs 2^21 bins (2 sweeps), 1 or 2 keys per lane.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/c5_shards.sh LSMB_SLICE_LOG2=20 && bash tools/c5_shards.sh LSMB_SLICE_LOG2=21 && \
  bash tools/c5_shards.sh LSMB_SLICE_LOG2=21 LSMB_SWEEP_PER=2
