cd ${GRAFT_REPO_ROOT:-/root/repo}
for fk in 100000000 84000000 112000000 100000000 84000000 112000000; do
  out=$(timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --filter-keys $fk --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-c1 --no-probe --no-c5 2>/dev/null) || { echo fail; exit 1; }
  echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; c=d["config"]; print("filter_keys %s num_bits %d bins %d pass_a %.4f pass_b %.4f" % (sys.argv[1], c["num_bits"], -(-c["num_bits"] // 2**20), r["pass_a_ms"], r["pass_b_ms"]))' $fk
done
