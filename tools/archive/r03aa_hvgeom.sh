#!/bin/bash
# C4 k_hash_var geometry A/B (one box): the product (256 keys / 36 KiB window,
# four workgroups per CU) against 512 keys / 72 KiB (two per CU, with and
# without a 4-waves-per-SIMD register cap) and 1024 keys / 144 KiB (one per CU).
# Variants built by tools/build_variants.sh with -DLSMB_HV_KEYS / _WIN / _WPE.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  bash tools/run_varlen_variants.sh base hv512 hv512w4 hv1024 || exit $?
done
