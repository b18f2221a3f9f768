# C5 shard with two keys per lane per phase forced (LSMB_SWEEP_PER=2; R=32 rings overflow more often into exact global atomics)
cd $GRAFT_REPO_ROOT
c5() { timeout -k 10 120 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 2 --no-probe --no-cpu-baseline --no-e2e --no-varlen --no-exact10 | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(sys.argv[1], "c5 pass_a %.4f pass_b %.4f kernel %.4f" % (r["pass_a_ms"], r["pass_b_ms"], r["kernel_ms"]), d.get("words_equal_oracle_fixture"))' "$1"; }
for rep in 1 2; do c5 per1 || exit $?; LSMB_SWEEP_PER=2 c5 per2 || exit $?; done
