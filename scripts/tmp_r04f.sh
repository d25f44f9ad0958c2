# round-4 batch: GPU tests, per-launch sweep (k_tail, shard counters), A/B of variants
set -e
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 scripts/launch_sweep.py scenes/spot.xml 8,16,64 tail:MFX_TAIL=1 notail:MFX_TAIL=0 "tail3:MFX_TAIL=1;MFX_TAIL_WAVES=3" "tail_t128:MFX_TAIL=1;MFX_TCHUNK=128" "hs1tail:MFX_SWEEP_LIB=build_variants/hs1.so;MFX_TAIL=1" > $O/sweep.txt 2>&1
cat $O/sweep.txt
for sc in spot.xml renault.xml cube_cornell.xml; do
  echo "== $sc" >> $O/ab.txt
  timeout -k 10 200 python3 scripts/ab_variants.py scenes/$sc 2 32 >> $O/ab.txt 2>&1
done
grep -E "==|SUMMARY" -A4 $O/ab.txt
