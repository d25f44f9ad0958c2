#!/bin/bash
# Bench lines for every BASELINE.json GPU config at N = 1 (C2 the metric's; C4/C5 one GPU's share
# of their 8-GPU workloads) plus the per-iteration diagnostic of C2. Run on the GPU box from the
# repo root: scripts/bench_configs.sh TAG
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/configs_$TAG
mkdir -p $OUT
for c in C2 C3 C4 C5; do
  timeout -k 10 300 python3 $R/bench.py --config $c --steps 2 --warmup 1 > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  cat $OUT/bench_$c.json
done
MFX_DIAG_ITER=1 timeout -k 10 120 python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stats \
  > $OUT/diag_iter_C2.json 2> $OUT/diag_iter_C2.err
