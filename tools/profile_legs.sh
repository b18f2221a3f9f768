#!/bin/bash
# Per-leg rocprofv3 passes (run through gpurun): every bench leg in a process of
# its own (tools/legs.py, 10 launches after its setup), each with a kernel trace
# (--stats) and separate --pmc passes (FETCH_SIZE; WRITE_SIZE; the SQ set and
# GRBM_GUI_ACTIVE).  tools/prof_summary.py --legs condenses them into
# profiles/traffic.json (read by bench.py: every leg's roofline.traffic and
# secondary ceilings).
# Usage: tools/profile_legs.sh <tag> [legs...]
set -uo pipefail
TAG=${1:-r04}; shift || true
LEGS=${*:-c2 exact10 c5 c5_full c4 probe fset fset_mixed fset_rows1}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/legs_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for leg in $LEGS; do
  mkdir -p "$OUT/$leg"
  for pass in stats fetch write sq; do
    case $pass in
      stats) a="--kernel-trace --stats" ;;
      fetch) a="--pmc FETCH_SIZE" ;;
      write) a="--pmc WRITE_SIZE" ;;
      sq) a="--pmc $SQ" ;;
    esac
    timeout -k 10 240 rocprofv3 $a --output-format csv -d "$OUT/$leg/$pass" -o run -- \
      python3 $REPO/tools/legs.py $leg --reps 10 > "$OUT/$leg/$pass.log" 2>&1
    rc=$?
    echo "$leg $pass rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 $REPO/tools/prof_summary.py "$OUT" --legs "$OUT/traffic.json" > "$OUT/legs_summary.md"
echo "profile $TAG done"
