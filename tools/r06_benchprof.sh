#!/bin/bash
# The default bench command under rocprofv3 --kernel-trace --stats (the
# contract's "same command": its per-kernel means against the line's event
# times), then the VALU issue-cost microbenchmark.  Each step time-limited.
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/${1:-r06e}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $REPO/bench.py --detail-out $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench under rocprof rc=$rc"; head -c 400 $OUT/bench.json; echo
[ $rc -eq 0 ] || exit $rc
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null || find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -12 $OUT/kernel_stats.csv
cd $REPO && timeout -k 10 120 ./tools/mb_valu > $OUT/valu_issue.jsonl 2>&1 || { echo "mb_valu failed"; exit 1; }
tail -3 $OUT/valu_issue.jsonl
