#!/bin/bash
# r02bl: the A/B of the scan-lookahead and node-loop-exit knobs after the cooperative sampler
# (build_variants/*.so). (The call's first version also ran the page-locked output A/B and the
# TD/TCP PMC passes: profiles/r02/r02bl_*.)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_ab.sh r02bl_ab 2 64 spot.xml renault.xml cube_cornell.xml
