#!/bin/bash
# Round-2 evidence on one box: pytest -m gpu, rocprof kernel stats + PMC traffic (C2, C5 two-level),
# bench lines C2-C5 (+ C5 flat). Output under gpurun_out/<tag>.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${1:-r02final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash scripts/profile_traffic.sh ${T}_c2 > /dev/null
bash scripts/profile_traffic.sh ${T}_c5 --config C5 > /dev/null
for c in C2 C3 C4 C5 C5F; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 > $O/bench_$c.json 2> $O/bench_$c.err
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', d['value'], d['ms_per_step'])"
done
