#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r01l
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01l/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01l/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/r01l/bench_default.json 2> gpurun_out/r01l/bench_default.err
cat gpurun_out/r01l/bench_default.json
bash scripts/bench_configs.sh r01l
cd /tmp && export TMPDIR=/tmp
for c in C3 C5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01l/trace_$c -o run -- \
    python3 $R/bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r01l/trace_$c.log 2>&1
done
