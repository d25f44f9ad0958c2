#!/bin/bash
# The TD (texture-data / vector-memory) roof of the trace kernels, in one rocprofv3 --pmc pass each
# (kernel trace on, no other trace domain): TCP_TOTAL_CACHE_ACCESSES (L1 tag lookups: one per line a
# wave memory instruction touches), TCP_TCC_READ_REQ (L1 misses), TD_TD_BUSY and GRBM_GUI_ACTIVE
# (GPU clocks per dispatch), on (1) the bench step and (2) the peak case of scripts/ubench/td_gather (every lane a
# distinct line of an L1-resident table). A second pass counts scalar-memory instructions
# (SQ_INSTS_SMEM, GRBM_GUI_ACTIVE) on the bench step and on scripts/ubench/sload's peak case (k_camera
# reads its nodes and slots through the scalar cache: its roof). scripts/summarize_td.py writes
# profiles/td_<scene>.json, which bench.py reads for roofline.td / roofline.smem.
# Usage: scripts/pmc_td_roof.sh TAG [extra bench args...]
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-td}
shift || true
OUT=$R/gpurun_out/tdroof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CTR="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $OUT/bench -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats --no-render-api "$@" > $OUT/bench.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $OUT/ubench -o run -- \
    $R/scripts/ubench/td_gather peak > $OUT/ubench.log 2>&1
SCTR="SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $SCTR --output-format csv -d $OUT/bench_smem -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats --no-render-api "$@" > $OUT/bench_smem.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SCTR --output-format csv -d $OUT/ubench_smem -o run -- \
    $R/scripts/ubench/sload peak > $OUT/ubench_smem.log 2>&1
python3 $R/scripts/summarize_td.py $OUT "$@"
