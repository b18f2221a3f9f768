#!/bin/bash
# Round-6 C4 k_hash_var geometry A/B on one box (more bytes
# in flight per CU): the product (256 keys / 36 KiB window, four workgroups per
# CU) against 128 keys / 18 KiB (eight per CU), 128 / 20 KiB (seven) and
# 192 / 27 KiB (five), all at <= 128 VGPRs; built by tools/build_variants.sh.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  bash tools/run_varlen_variants.sh base hv128 hv128w20 hv192 || exit $?
done
