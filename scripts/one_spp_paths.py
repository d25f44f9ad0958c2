"""1-spp render calls (Scene.Render without render-ahead): megakernel vs wavefront, mfx_render_rgba8 per call
(bench.render_api) on three scenes. Usage: python3 scripts/one_spp_paths.py (GPU box)."""
import sys, os, json
sys.path.insert(0, os.getcwd())
import bench
from mafrixraytracing_amd.abi import MFX_F_WAVEFRONT
from mafrixraytracing_amd.native import DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
for sc in ["spot.xml", "renault.xml", "cube_cornell.xml"]:
    a = load_scene_file("scenes/" + sc)
    for fl, lab in [(0, "mega"), (MFX_F_WAVEFRONT, "wavefront")]:
        r = bench.render_api(a, DEFAULT_SEED, 64, flags=fl)
        print(sc, lab, round(r["value"], 1), r["ms_per_call"], r["trace_device_ms_per_call"], flush=True)
