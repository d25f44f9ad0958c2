#!/bin/bash
# TD / TCP / SQ memory-pipeline counters of the wavefront kernels, the groups of round 1's
# profiles/r01b_pmc_td_tcp_utcl1.txt (one rocprofv3 --pmc pass per group), on the C2 bench step.
# Usage: scripts/pmc_td.sh TAG [extra bench args...]
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-td}
shift || true
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_ACCESSES_sum TCP_TCP_LATENCY_sum TCP_TA_TCP_STATE_READ_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats --no-render-api "$@" > $OUT/p$i.log 2>&1 \
      || { echo "pass $i failed" >> $OUT/errors.txt; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
with open(out + "/summary.txt", "w") as fo:
    for k, d in agg.items():
        if "k_" not in k:
            continue
        fo.write(k + "\n")
        for c, v in sorted(d.items()):
            fo.write(f"  {c} {v:.4g}\n")
print(open(out + "/summary.txt").read())
PY
