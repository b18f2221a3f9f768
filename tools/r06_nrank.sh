#!/bin/bash
# Round-6 full-size N > 1 rehearsal on one GPU (ranks share the card, so the
# numbers are not scaling; the path, its checks and the step forms are what
# is exercised): C5, 1e9 keys, --gpus 2 / 4 / 8 with the IPC merge.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r06q}
mkdir -p $OUT
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --gpus $n --backend ipc --no-cpu-baseline \
    --detail-out $OUT/n${n}_detail.json > $OUT/n${n}.json 2> $OUT/n${n}.err
  rc=$?
  echo "n=$n rc=$rc"
  head -c 400 $OUT/n${n}.json; echo
  [ $rc -eq 0 ] || exit $rc
done
