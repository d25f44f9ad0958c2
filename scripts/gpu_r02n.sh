#!/bin/bash
# r02n: rocprof kernel stats + PMC HBM traffic (FETCH_SIZE x2, WRITE_SIZE; separate passes) of the
# C2 bench and C5, and the render-API (Scene.Render pattern) kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/profile_traffic.sh r02n_c2 > /dev/null
bash scripts/profile_traffic.sh r02n_c5 --config C5 > /dev/null
O=$R/gpurun_out/prof_r02n_render
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --api render --no-cpu-baseline --no-stats --steps 1 --warmup 1 > $O/bench.log 2>&1
ls $R/gpurun_out/prof_r02n_c2 $R/gpurun_out/prof_r02n_c5
