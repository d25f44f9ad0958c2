#!/bin/bash
# r02bo: instance frame switches re-origin the FP32 ray (no divisions): pytest -m gpu with the
# in-tree build, then A/B against the previous tree (build_variants/*.so) on C5 two-level and C2
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02bo
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
bash scripts/gpu_ab.sh r02bo_ab 3 64 spot16_instanced.xml spot.xml
