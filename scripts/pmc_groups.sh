#!/bin/bash
# One rocprofv3 --pmc pass per counter group on the bench workload; summary per kernel.
# Usage: scripts/pmc_groups.sh TAG "GROUP1" "GROUP2" ...
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/errors.txt; exit 1; }
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
