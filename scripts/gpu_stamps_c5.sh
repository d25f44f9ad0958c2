#!/bin/bash
# Phase stamps (k_extend st1, k_shadow st2) on the C5 scene, two-level vs flat: gpurun_out/$1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/${1:-stamps}
mkdir -p $OUT
for v in st1 st2; do
  for sc in spot16_instanced spot16; do
    timeout -k 10 200 python3 scripts/diag_stamps.py build_variants/$v.so scenes/$sc.xml 8 >> $OUT/stamps.txt 2>&1
    echo "$v $sc" >> $OUT/stamps.txt
  done
done
cat $OUT/stamps.txt
