#!/bin/bash
# C5 two-level vs flat A/B bench lines (no render_api / CPU legs). Output under gpurun_out/$1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/${1:-c5ab}
mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -u -m pytest $2 -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
fi
for c in C5 C5F; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-render-api > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['stage_ms']['extend_ms'], r['stage_ms']['shadow_ms'])"
done
