#!/bin/bash
# A/B of pass B (k_apply): the product's one-region-at-a-time loads against
# the next chunk's loads in flight during the apply (LSMB_APPLY_PIPE=1, variant
# "pipe") and a loads-only ablation ("ldonly", LSMB_ABL=32: no LDS ORs, wrong
# filters by construction).  Built by
#   tools/build_variants.sh pipe="-DLSMB_APPLY_PIPE=1" ldonly="-DLSMB_ABL=32"
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
bash tools/run_variants.sh --no-c1 --no-probe -- base pipe ldonly base pipe ldonly
