#!/bin/bash
# Pass B region loads with (product) and without (liblsmbloom_plain.so) the
# non-temporal hint: C5's two half-bin workgroups read every region of their
# bin, so the second read may hit L2 more often without it.  C2 + C5 shard,
# two repetitions, plus rocprofv3 kernel stats of the C5 leg each way.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/r04plain
mkdir -p $OUT
L=$PWD/storage-engine_amd/lib
one() {  # tag lib
  LSMB_LIB=$2 timeout -k 10 180 python3 bench.py --steps 20 --warmup 10 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 \
    --no-probe --no-c1 > $OUT/$1.json 2> $OUT/$1.err || return $?
  LSMB_LIB=$2 timeout -k 10 180 python3 bench.py --global-keys 125000000 --filter-keys 1000000000 --steps 10 --warmup 5 \
    --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-probe --no-c1 > $OUT/$1_c5.json 2>> $OUT/$1.err || return $?
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); e=json.load(open(sys.argv[2])); r=d["roofline"]; q=e["roofline"]; print("%-7s C2 kernel %.4f pass_b %.4f exact %s | C5 kernel %.4f pass_a %.4f pass_b %.4f" % (sys.argv[3], r["kernel_ms"], r["pass_b_ms"], d.get("words_equal_oracle_fixture"), q["kernel_ms"], q["pass_a_ms"], q["pass_b_ms"]))' $OUT/$1.json $OUT/$1_c5.json $1
}
for rep in 1 2; do
  one nt_$rep $L/liblsmbloom.so || exit $?
  one plain_$rep $L/liblsmbloom_plain.so || exit $?
done
