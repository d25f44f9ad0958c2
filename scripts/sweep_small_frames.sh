#!/bin/bash
# Chunk sizes for the strong-scaling shares with frames in flight: scripts/frames_in_flight.py at
# the 1/8 and 1/4 shares of C2 with 2 and 3 contexts, per environment setting (one line each).
# Usage: scripts/sweep_small_frames.sh TAG "ENV=V ..." ...   (an empty string: the defaults)
set -e
O=gpurun_out/$1; shift
mkdir -p $O
for e in "$@"; do
  echo "== ${e:-defaults}" >> $O/sweep.txt
  env $e timeout -k 10 120 python3 scripts/frames_in_flight.py --parts 8,4 --modes 2,3 --steps 12 >> $O/sweep.txt 2>> $O/sweep.err
done
cat $O/sweep.txt
