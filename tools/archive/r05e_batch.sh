mkdir -p gpurun_out
bash tools/run_variants.sh --no-probe --no-c1 -- base permjob abl1 abl8 abl16 base permjob > gpurun_out/r05e_abl.log 2>&1 || exit $?
cat gpurun_out/r05e_abl.log
LSMB_LIB=storage-engine_amd/lib/liblsmbloom_stamp.so timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-probe --no-c1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 > /dev/null 2> gpurun_out/r05e_stamp.err || exit $?
grep stamp gpurun_out/r05e_stamp.err | tail -2
(cd tools && hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_mall.hip -o /tmp/mb_mall 2>/dev/null) || exit 3
timeout -k 10 200 /tmp/mb_mall > gpurun_out/r05e_mall.jsonl 2>&1 || exit $?
timeout -k 10 200 python3 tools/probe_scale.py > gpurun_out/r05e_probe_scale.jsonl 2>&1 || exit $?
tail -2 gpurun_out/r05e_probe_scale.jsonl
