#!/bin/bash
# A/B of build_variants/*.so (gpu_ab.sh) followed by an MFX_DIAG_ITER run of the tree's library on C2
# gpu_ab_diag.sh TAG ROUNDS SPP scene1.xml [...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_ab.sh "$@"
