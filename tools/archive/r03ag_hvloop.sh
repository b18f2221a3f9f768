#!/bin/bash
# Variant sources: tools/r03_hvloop.patch applied to a copy of csrc/ (hash_var.hip built with
# -DLSMB_HV_WGS_PER_CU=4|0 and with or without -mllvm -disable-machine-licm).
# C4 k_hash_var block loop (next block's bounds prefetched by LDS-DMA), built in
# a scratch tree (not the product): grid capped at 4 workgroups per CU (l4*) or
# one block per workgroup (l0*), with (l*l) or without (l*n) MachineLICM in the
# k_hash_var translation unit; against the product (base).  Separates the loop's
# cost from the codegen flag's.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  bash tools/run_varlen_variants.sh base l4n l0n l4l l0l || exit $?
done
