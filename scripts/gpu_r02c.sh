#!/bin/bash
# r02c: default bench line (with render_api + cpu_baseline strict/fast), the render-API headline,
# single-process device-list path, strong scaling mode at N=1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python3 bench.py --api render --no-cpu-baseline --steps 2 > $O/bench_render.json 2> $O/bench_render.err
timeout -k 10 300 python3 bench.py --single-process --gpus 1 --no-cpu-baseline --no-render-api > $O/bench_single.json 2> $O/bench_single.err
timeout -k 10 300 python3 bench.py --scaling strong --no-cpu-baseline --no-render-api > $O/bench_strong.json 2> $O/bench_strong.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_render -o run -- \
    python3 $R/bench.py --api render --no-cpu-baseline --no-stats --steps 1 --warmup 1 > $R/$O/trace_render.log 2>&1
cat $R/$O/bench_default.json $R/$O/bench_render.json
