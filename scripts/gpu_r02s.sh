#!/bin/bash
# Round 2 (s): instancing parity + C5 two-level vs flat bench lines. Output under gpurun_out/r02s.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/r02s
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_instancing.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_inst.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_build.py -k "spot16_instanced" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_parity_inst.log 2>&1
for c in C5 C5F; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  cat $OUT/bench_$c.json
done
