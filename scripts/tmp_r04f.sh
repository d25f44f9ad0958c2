mkdir -p gpurun_out/r04f
timeout -k 10 500 python3 scripts/launch_sweep.py scenes/spot.xml 8,16,64 tail:MFX_TAIL=1 notail:MFX_TAIL=0 "tail3:MFX_TAIL=1;MFX_TAIL_WAVES=3" "tail_t128:MFX_TAIL=1;MFX_TCHUNK=128" "hs1tail:MFX_SWEEP_LIB=build_variants/hs1.so;MFX_TAIL=1" "hs1notail:MFX_SWEEP_LIB=build_variants/hs1.so;MFX_TAIL=0" > gpurun_out/r04f/sweep.txt 2>&1
cat gpurun_out/r04f/sweep.txt
