#!/bin/bash
# r02bv: the final tree (after the derived keys): pytest -m gpu, smoke, the default bench line (what the driver runs).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02bv
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
