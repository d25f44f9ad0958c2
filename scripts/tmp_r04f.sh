# round-4 batch: per-launch sweep (k_tail), A/B of the chunk-counter variants
set -e
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 python3 scripts/launch_sweep.py scenes/spot.xml 8,16,64 tail:MFX_TAIL=1 notail:MFX_TAIL=0 "tail3:MFX_TAIL=1;MFX_TAIL_WAVES=3" > $O/sweep.txt 2>&1 || true
cat $O/sweep.txt
for sc in spot.xml renault.xml cube_cornell.xml; do
  echo "== $sc" >> $O/ab.txt
  timeout -k 10 250 python3 scripts/ab_variants.py scenes/$sc 2 32 >> $O/ab.txt 2>&1
done
grep -E "==|SUMMARY" $O/ab.txt
