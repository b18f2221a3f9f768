#!/bin/bash
# Round-6 end-of-round rehearsal (the driver's order): the -m gpu suite,
# smoke(), then the default bench line.  Stops at the first step that fails
# (a pytest failure too); each step has its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r06f}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; head -c 300 $OUT/bench.json; echo
exit $rc
