#!/bin/bash
# SQ / TCP / TCC counter passes for the trace kernel (one rocprofv3 --pmc pass per group).
# bench.py refuses to relaunch itself under rocprofv3: the hardware queues come from here
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${1:-r01}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/errors.txt
done
for f in $OUT/p*/run_counter_collection.csv; do grep -h trace_kernel $f | awk -F'","' '{print $0}' | sed 's/.*"\(SQ_[A-Z_]*\|TCC_[A-Za-z_]*\|TCP_[A-Za-z_]*\|GRBM_[A-Z_]*\)",\([0-9.e+]*\).*/\1 \2/' ; done > $OUT/summary.txt
cat $OUT/summary.txt
