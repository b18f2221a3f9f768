cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r02n}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG:-r02n}_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r02n}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG:-r02n}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG:-r02n}_bench.json 2> gpurun_out/${TAG:-r02n}_bench.err
echo "bench rc=$?"
