# C5 shard and C4: current library vs the round-2 kernels (433247d), C5 keys-per-lane knob
cd $GRAFT_REPO_ROOT
R2=$PWD/storage-engine_amd/lib/liblsmbloom_r2.so
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "pass_a %.4f pass_b %.4f kernel %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]))' "$1"; }
c4() { timeout -k 10 180 python3 bench.py --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline())["varlen"]; print(sys.argv[1], "pass_a %.4f pass_b %.4f kernel %.4f frac %.4f" % (d["pass_a_ms"], d["pass_b_ms"], d["kernel_ms"], d["frac"]), d.get("words_equal_oracle_fixture"))' "$1"; }
for rep in 1 2; do c5 cur || exit $?; LSMB_LIB=$R2 c5 r2 || exit $?; done
LSMB_SWEEP_PER=1 c5 cur_per1 || exit $?
LSMB_SWEEP_PER=1 LSMB_LIB=$R2 c5 r2_per1 || exit $?
c4 cur || exit $?; LSMB_LIB=$R2 c4 r2 || exit $?
