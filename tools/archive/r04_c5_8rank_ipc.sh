#!/bin/bash
# The N = 8 C5 step with the cross-process peer-load merge (--backend ipc):
# 8 rank processes on the one GPU (125 M keys each into the 2^32-1-bit
# filter, two sweeps, each sweep's range merged by IPC peer loads while the
# next builds).  RCCL refuses ranks sharing a device; IPC does not, so this
# runs the product merge of the N > 1 path end to end: rank 0 checks the merged
# words against the oracle's full-size C5 digest and against its own
# single-process rebuild.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04c5}
mkdir -p gpurun_out/$TAG
( while sleep 30; do echo tick $(date +%T); done ) &
TICK=$!
timeout -k 10 600 python3 bench.py --gpus 8 --backend ipc --steps 2 --warmup 1 --no-probe --no-cpu-baseline --no-e2e \
  --no-varlen --no-exact10 > gpurun_out/$TAG/c5_8rank_ipc.json 2> gpurun_out/$TAG/c5_8rank_ipc.err
rc=$?
kill $TICK
echo "8rank ipc rc=$rc"
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print({k: d.get(k) for k in ("n_gpus", "value", "ms_per_step", "words_equal_oracle_fixture", "multi_gpu_merged_equals_single_gpu_build")}, d["step_split"])' gpurun_out/$TAG/c5_8rank_ipc.json
exit $rc
