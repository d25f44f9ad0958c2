#!/bin/bash
# VALU / FP64 instruction mix and wave activity of the trace kernels on the C2 bench step (two
# rocprofv3 --pmc passes of 8 counters each, kernel trace on) -> gpurun_out/r04y/summary.txt
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04y
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats --no-render-api"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 $B > $OUT/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $OUT/p2 -o run -- python3 $B > $OUT/p2.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add((f, r["Dispatch_Id"]))
with open(out + "/summary.txt", "w") as fo:
    for k, d in agg.items():
        if "k_" not in k:
            continue
        fo.write(f"{k} (dispatches over passes: {len(n[k])})\n")
        for c, v in sorted(d.items()):
            fo.write(f"  {c} {v:.4g}\n")
print(open(out + "/summary.txt").read())
PY
