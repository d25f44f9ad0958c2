#!/bin/bash
# r02bu: k_extend's ray counters per wave (MFX_WAVE_COUNTERS) A/B, build_variants/*.so
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_ab.sh r02bu_ab 3 64 spot.xml renault.xml cube_cornell.xml
