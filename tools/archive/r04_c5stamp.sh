#!/bin/bash
# C5 shard pass A phase sections (LSMB_STAMP build of this tree, fresh sweeps):
# where the sweep's phase goes now that the saturated filter walks by folding.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04cs
L=$PWD/storage-engine_amd/lib
LSMB_LIB=$L/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 \
  --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 \
  > gpurun_out/r04cs/c5.json 2> gpurun_out/r04cs/c5.err || exit $?
grep stamp gpurun_out/r04cs/c5.err | tail -2
LSMB_LIB=$L/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline \
  --no-varlen --no-exact10 --no-probe --no-c1 > gpurun_out/r04cs/c2.json 2> gpurun_out/r04cs/c2.err || exit $?
grep stamp gpurun_out/r04cs/c2.err | tail -1
