#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
bash scripts/profile_traffic.sh r02q_c2 > /dev/null
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
