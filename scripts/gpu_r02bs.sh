#!/bin/bash
# r02bs: camera-ray path keys derived in k_shadow instead of stored by k_extend (MFX_KEY_RECOMPUTE) A/B
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_ab.sh r02bs_ab 3 64 spot.xml renault.xml cube_cornell.xml
