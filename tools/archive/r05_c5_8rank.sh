#!/bin/bash
# The N = 8 C5 step on the one GPU: 8 rank processes (125 M keys each into the
# 2^32-1-bit filter, two sweeps), merged by the device-ordered IPC peer loads
# (--backend ipc) or by auto's two-merge path with gloo in RCCL's place
# (--backend auto-gloo: both merges set up, checked against each other, the
# faster timed).  Not a scaling figure (8 ranks share one GPU): the point is
# the N > 1 code path end to end, with rank 0 checking the merged words against
# the oracle's full-size C5 digest and its own single-process rebuild.
# Usage: tools/r05_c5_8rank.sh <tag> <backend>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r05c5}; BK=${2:-ipc}
mkdir -p gpurun_out/$TAG
( while sleep 30; do echo tick $(date +%T); done ) &
TICK=$!
timeout -k 10 600 python3 bench.py --gpus 8 --backend $BK --steps 2 --warmup 1 --no-probe --no-cpu-baseline --no-e2e \
  --no-varlen --no-exact10 > gpurun_out/$TAG/c5_8rank_$BK.json 2> gpurun_out/$TAG/c5_8rank_$BK.err
rc=$?
kill $TICK
echo "8rank $BK rc=$rc"
python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); print({k: d.get(k) for k in ("n_gpus", "value", "ms_per_step", "words_equal_oracle_fixture", "multi_gpu_merged_equals_single_gpu_build")}, d["step_split"])' gpurun_out/$TAG/c5_8rank_$BK.json
exit $rc
