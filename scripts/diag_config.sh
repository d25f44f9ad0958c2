mkdir -p gpurun_out/r06cfg
for sc in spot renault spot16_instanced; do
MFX_DIAG_ITER=1 timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
from mafrixraytracing_amd.native import NativeContext
from mafrixraytracing_amd.scene_io import load_scene_file
a=load_scene_file('scenes/$sc.xml')
with NativeContext(a, seed=1) as c:
    c.trace_accumulate(1,0); c.sync()
" 2>&1 | grep -m1 "top nodes in LDS" | sed "s/^/$sc: /" >> gpurun_out/r06cfg/cfg.txt
done
cat gpurun_out/r06cfg/cfg.txt
