#!/bin/bash
# r02bn: k_resolve's first-round loads (WF_RES_EAGER 0 / 1 / 2) A/B, build_variants/*.so
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_ab.sh r02bn_ab 3 64 spot.xml renault.xml cube_cornell.xml
