#!/bin/bash
# Per-iteration stage times (MFX_DIAG_ITER) of build_variants/*.so, each with its .env, on one scene:
# scripts/diag_ab.sh TAG SCENE SPP. Output gpurun_out/TAG/diag_ab.txt.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/$1; mkdir -p $O
for round in 0 1; do
  for l in build_variants/*.so; do
    E=(); [ -f ${l%.so}.env ] && E=($(cat ${l%.so}.env))
    env "${E[@]}" timeout -k 10 120 python3 scripts/diag_variant.py $l scenes/$2 $3 >> $O/diag_ab.txt 2>&1
  done
done
grep -E "^---|gen 0 iter|\{'total" $O/diag_ab.txt | grep -v "trace 0" | grep -A4 -E "^---" > $O/diag_ab_summary.txt || true
cat $O/diag_ab_summary.txt
