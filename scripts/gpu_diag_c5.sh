set -e
mkdir -p gpurun_out/r02v
for c in C5 C5F; do
MFX_DIAG_ITER=1 timeout -k 10 200 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-stats --no-render-api > gpurun_out/r02v/diag_$c.json 2> gpurun_out/r02v/diag_$c.err
done
