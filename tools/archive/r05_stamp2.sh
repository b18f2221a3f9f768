cd ${GRAFT_REPO_ROOT:-/root/repo}
for v in st st2 st st2; do
  LSMB_LIB=$PWD/storage-engine_amd/lib/liblsmbloom_$v.so timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-varlen --no-exact10 --no-c1 --no-probe --no-c5 2>&1 >/dev/null | grep stamp | tail -2 | sed "s/^/$v /"
done
