cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r02k_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02k_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r02k_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r02k_bench.json 2> gpurun_out/r02k_bench.err
echo "bench rc=$?"
