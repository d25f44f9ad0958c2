#!/bin/bash
# Bench lines (no render_api / CPU legs) for the configs given after the tag: gpurun_out/<tag>/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in "$@"; do
  env ${DIAG:+MFX_DIAG_ITER=1} timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-render-api > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['stage_ms']['extend_ms'], r['stage_ms']['shadow_ms'])"
done
