#!/bin/bash
# pytest -m gpu (whole suite), then the default bench line (render_api with and without render-ahead)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${1:-r02az}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 > $O/bench_default.json 2> $O/bench_default.err
python3 -c "import json; d=json.load(open('$O/bench_default.json')); r=d['render_api']; print(d['value'], d['ms_per_step'], r['value'], r['ms_per_call'], r['with_render_ahead']['value'], r['with_render_ahead']['ms_per_call'], r['with_render_ahead']['ms_per_call_max'])"
