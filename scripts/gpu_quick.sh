#!/bin/bash
# Quick GPU check of the tree: pytest -m gpu, smoke, default bench line. Output under gpurun_out/$1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-quick}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err
cat gpurun_out/$TAG/bench_default.json
