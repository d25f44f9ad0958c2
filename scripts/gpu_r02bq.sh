#!/bin/bash
# r02bq: k_resolve register budget (WF_RES_WAVES 6 / 8, WF_RES_VERTS 2) A/B, build_variants/*.so
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_ab.sh r02bq_ab 2 64 spot.xml cube_cornell.xml
