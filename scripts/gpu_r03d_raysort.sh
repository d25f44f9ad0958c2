set -e
O=gpurun_out/r03d; mkdir -p $O
MFX_RAY_SORT=1 MFX_RAY_SORT_OBITS=2 MFX_RAY_SORT_DBITS=6 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "image_parity or full_frame or partitions" > $O/pytest_raysort.log 2>&1
tail -1 $O/pytest_raysort.log
for cfg in "0 0 3" "1 4 3" "1 0 6" "1 2 6"; do set -- $cfg
  MFX_DIAG_ITER=1 MFX_RAY_SORT=$1 MFX_RAY_SORT_OBITS=$2 MFX_RAY_SORT_DBITS=$3 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-render-api --no-stats > $O/diag_$1_$2_$3.json 2> $O/diag_$1_$2_$3.txt
done
bash scripts/gpu_run.sh r03d ab:2:64:spot.xml,renault.xml,cube_cornell.xml
