#!/bin/bash
# Round-end rehearsal: the whole -m gpu suite, smoke(), then the default bench line (as the driver runs it).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${1:-r03z}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${1:-r03z}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 400 python bench.py > gpurun_out/${1:-r03z}_bench.json 2> gpurun_out/${1:-r03z}_bench.err || exit $?
python3 -c 'import json; d=json.load(open("gpurun_out/'${1:-r03z}'_bench.json")); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r.get("traffic"), r.get("traffic_stale"), d.get("words_equal_oracle_fixture"))'
exit $rc
