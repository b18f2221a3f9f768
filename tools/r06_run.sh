#!/bin/bash
# Round-6 GPU call: [optional MALL microbenchmark] + the -m gpu tests (all, or
# a -k expression) + the default bench line.  Test failures (pytest rc 1)
# still let the bench run; a timeout / abort / segfault ends the call.
# Usage: tools/r06_run.sh <tag> [pytest -k expr | all | none] [mall]
TAG=${1:-r06}
K=${2:-all}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$3" = "mall" ]; then
  timeout -k 10 240 ./tools/mb_mall > $OUT/mall.jsonl 2> $OUT/mall.err
  rc=$?
  echo "mall rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 120 ./tools/mb_lds > $OUT/lds.log 2>&1
  rc=$?
  echo "lds rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "$K" != "none" ]; then
  if [ "$K" = "all" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  else
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
  fi
  rc=$?
  echo "tests rc=$rc"
  tail -5 $OUT/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py --detail-out $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err
brc=$?
echo "bench rc=$brc"
head -c 600 $OUT/bench.json
exit $brc
