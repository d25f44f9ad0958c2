#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
# 1) kernel trace + stats of the bench command; 2) FETCH_SIZE; 3) WRITE_SIZE (separate --pmc
# passes: the two counters do not fit one TCC pass on gfx950). Then summarise into
# $OUT/traffic.json (per-kernel HBM bytes per launch, gfx950 FETCH_SIZE correction applied).
# Usage: scripts/profile_traffic.sh TAG [extra bench args...]
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
shift || true
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render-api "$@" > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats --no-render-api "$@" > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats --no-render-api "$@" > $OUT/bench_write.log 2>&1
python3 $R/scripts/summarize_profile.py $OUT "$@"
