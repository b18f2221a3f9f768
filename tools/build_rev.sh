#!/bin/bash
# A/B helper (tools only): builds the library as of git revision REV into
# storage-engine_amd/lib/liblsmbloom_NAME.so, so one GPU call can time both
# sides on the same box (tools/run_variants.sh ... -- base NAME).
# Usage: tools/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/lsmb_rev_$NAME
rm -rf "$WT"
git -C "$ROOT" worktree add -f --detach "$WT" "$REV" >/dev/null 2>&1
make -C "$WT/storage-engine_amd" -j8 lib/liblsmbloom.so >/dev/null
cp "$WT/storage-engine_amd/lib/liblsmbloom.so" "$ROOT/storage-engine_amd/lib/liblsmbloom_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $NAME from $(git -C "$ROOT" rev-parse --short "$REV")"
