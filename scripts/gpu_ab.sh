#!/bin/bash
# A/B of build_variants/*.so on scenes (ab_variants.py, one process per variant, interleaved):
# gpu_ab.sh TAG ROUNDS SPP scene1.xml [scene2.xml ...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$1; ROUNDS=$2; SPP=$3; shift 3
mkdir -p gpurun_out/$TAG
for sc in "$@"; do
  echo "== $sc" >> gpurun_out/$TAG/ab.txt
  timeout -k 10 900 python3 scripts/ab_variants.py scenes/$sc $ROUNDS $SPP >> gpurun_out/$TAG/ab.txt 2>&1
done
grep -E "==|SUMMARY" gpurun_out/$TAG/ab.txt
