#!/bin/bash
# pytest -m gpu on the tree's library, then an A/B of build_variants/*.so (gpu_ab.sh):
# gpu_test_ab.sh TAG ROUNDS SPP scene1.xml [...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$1
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
tail -1 gpurun_out/$TAG/pytest_gpu.log
bash scripts/gpu_ab.sh "$@"
