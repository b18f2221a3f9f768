#!/bin/bash
# Round-6 A/B (one box): pass B of 2^21-bit bins with other-half offsets ORing a
# zero mask, all lanes active (product, LSMB_APPLY_ZMASK=1) vs the exec-masked
# form (zm0).  Parity first (the 2^21-bit-bin tests with the product library),
# then the C5 shard leg of bench.py, alternating, two reps each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r06b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fresh.py tests/test_gpu_random.py \
  -m gpu -v --timeout 300 --timeout-method thread -k "sweep or c5 or huge or random or fresh or slice" > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base zm0; do
    lib=storage-engine_amd/lib/liblsmbloom_$v.so; [ $v = base ] && lib=storage-engine_amd/lib/liblsmbloom.so
    LSMB_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 5 --no-probe --no-e2e --no-cpu-baseline \
      --no-varlen --no-exact10 --no-c1 --no-c5-full --detail-out $OUT/detail_$v.json > $OUT/b_$v.json 2> $OUT/b_$v.err || { echo "bench $v failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b_$v.json')); c=d['legs']['c5_shard']; r=d['roofline']
print('$v rep $rep c5_shard kernels %.4f pass_a %.4f pass_b %.4f exact %s | C2 kernels %.4f pass_b %.4f exact %s' % (c['kernel_ms'], c['pass_a_ms'], c['pass_b_ms'], c['words_equal_oracle_fixture'], r['kernel_ms'], r['pass_b_ms'], d.get('words_equal_oracle_fixture')))" | tee -a $OUT/ab.log
  done
done
