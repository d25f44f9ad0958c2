#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 300 python3 bench.py --api render --no-cpu-baseline --steps 2 > $O/bench_render.json 2> $O/bench_render.err
timeout -k 10 300 python3 bench.py --api render --megakernel --no-cpu-baseline --steps 2 > $O/bench_render_mega.json 2> $O/bench_render_mega.err
timeout -k 10 300 python3 bench.py --single-process --gpus 1 --no-cpu-baseline --no-render-api > $O/bench_single.json 2> $O/bench_single.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-render-api > $O/bench_default.json 2> $O/bench_default.err
for f in bench_render bench_render_mega bench_single bench_default; do python3 -c "import json,sys; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'])"; done
