#!/bin/bash
# One GPU call: the -m gpu suite, then (unless the suite crashed / hung) a
# short bench.  A pytest exit of 1 (test failures) still lets the bench run;
# a timeout (124/137), abort (134) or segfault (139) ends the call.
# Usage: tools/gpu_check.sh <tag> [pytest -k expr]
TAG=${1:-chk}
K=${2:-}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=3 -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=3 -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
fi
rc=$?
echo "tests rc=$rc"
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
brc=$?
echo "bench rc=$brc"
exit $brc
