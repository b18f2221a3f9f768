#!/bin/bash
# Round-6 A/B (one box): pass A's cooperative flush with two lanes per 64-B
# segment, one round of 32 jobs (LSMB_FLUSH_LANES=2, library "f2"), against
# the product's four lanes in two rounds.  Parity of the variant first (the
# partition / sweep / randomized / fresh GPU tests through LSMB_LIB), then
# C2 + the C5 shard, alternating, three reps each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r06d}
V=${2:-f2}
mkdir -p $OUT
LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_$V.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_fresh.py tests/test_gpu_random.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/parity_$V.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity_$V.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base $V; do
    lib=storage-engine_amd/lib/liblsmbloom_$v.so; [ $v = base ] && lib=storage-engine_amd/lib/liblsmbloom.so
    LSMB_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 10 --no-probe --no-e2e --no-cpu-baseline \
      --no-varlen --no-exact10 --no-c1 --no-c5-full --detail-out $OUT/detail_$v.json > $OUT/b_$v.json 2> $OUT/b_$v.err || { echo "bench $v failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b_$v.json')); c=d['legs']['c5_shard']; r=d['roofline']
print('%-5s rep $rep C2 kernels %.4f pass_a %.4f pass_b %.4f step %.4f exact %s | c5_shard kernels %.4f pass_a %.4f pass_b %.4f exact %s' % ('$v', r['kernel_ms'], r['pass_a_ms'], r['pass_b_ms'], d['ms_per_step'], d.get('words_equal_oracle_fixture'), c['kernel_ms'], c['pass_a_ms'], c['pass_b_ms'], c['words_equal_oracle_fixture']))" | tee -a $OUT/ab.log
  done
done
