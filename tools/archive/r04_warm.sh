#!/bin/bash
# C2 headline vs warmup length on one box (the GPU clock ramps over the first
# milliseconds of back-to-back work): --warmup 5 (the old default), 20, 40.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04w
for rep in 1 2; do
  for w in 5 20 40; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup $w --no-e2e --no-cpu-baseline --no-varlen --no-exact10 \
      --no-probe --no-c1 > gpurun_out/r04w/w$w.json 2>/dev/null || exit $?
    python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("warmup %-3s step %.4f ms kernels %.4f value %.0f" % (sys.argv[2], d["ms_per_step"], d["roofline"]["kernel_ms"], d["value"]))' gpurun_out/r04w/w$w.json $w
  done
done
