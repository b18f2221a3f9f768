#!/bin/bash
# 64-B vs 128-B segment slots (LSMB_SEG_STRIDE=128: every segment alone in its 128-B line), fresh builds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=$PWD/storage-engine_amd/lib
LSMB_LIB=$D/liblsmbloom_seg128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fresh.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03y_tests.log 2>&1
rc=$?; echo "seg128 fresh tests rc=$rc"; tail -1 gpurun_out/r03y_tests.log; [ $rc -ne 0 ] && exit $rc
summ='import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print("%-12s step %.4f pass_a %.4f pass_b %.4f kernel %.4f" % (sys.argv[1], d["ms_per_step"], r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))'
B="--no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 --no-c1"
c2() { timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 $B | python3 -c "$summ" "$1"; }
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 $B | python3 -c "$summ" "$1"; }
for rep in 1 2; do
  c2 c2_seg64 || exit $?
  LSMB_LIB=$D/liblsmbloom_seg128.so c2 c2_seg128 || exit $?
  c5 c5_seg64 || exit $?
  LSMB_LIB=$D/liblsmbloom_seg128.so c5 c5_seg128 || exit $?
done
cd /tmp && export TMPDIR=/tmp
for L in liblsmbloom.so liblsmbloom_seg128.so; do
  for C in FETCH_SIZE WRITE_SIZE; do
    LSMB_LIB=$D/$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03y_${L%.so}_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 $B > /dev/null 2>&1 || exit $?
  done
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections
for L in ("liblsmbloom", "liblsmbloom_seg128"):
    for C in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob("gpurun_out/r03y_%s_%s/run_counter_collection.csv" % (L, C))
        v = collections.defaultdict(list)
        for r in csv.DictReader(open(f[0])):
            if r["Kernel_Name"].startswith(("lsmb::(anonymous namespace)::k_bin", "lsmb::(anonymous namespace)::k_apply", "void lsmb::(anonymous namespace)::k_bin", "void lsmb::(anonymous namespace)::k_apply")):
                v[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
        for k, x in v.items():
            print(L, C, k, "%.1f MB" % ((2 if C == "FETCH_SIZE" else 1) * sum(x) / len(x) * 1024 / 1e6))
PY
