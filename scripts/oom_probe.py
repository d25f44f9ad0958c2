#!/usr/bin/env python3
"""How much free device memory a trace needs beside its path pool: a context created with room,
then all but `left` GB of the device taken by a torch allocation, then one C2 trace with a fixed
pool (MFX_POOL paths). Prints, per setting, whether the trace ran and the free memory around it."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(os.path.join(ROOT, "scenes", "spot.xml"))
    out = []
    for left_gb, spp in ((16, 8), (8, 8), (4, 8), (2, 8), (1, 8), (8, 64)):
        ctx = NativeContext(a, seed=DEFAULT_SEED)
        free0, _ = torch.cuda.mem_get_info()
        hog = torch.empty(max(0, free0 - (left_gb << 30)), dtype=torch.uint8, device="cuda")
        free1, _ = torch.cuda.mem_get_info()
        err = None
        try:
            ctx.trace_accumulate(spp, 0)
            ctx.sync()
        except Exception as e:  # noqa: BLE001 (the probe reports it)
            err = str(e)[-160:]
        free2, _ = torch.cuda.mem_get_info()
        del hog
        torch.cuda.empty_cache()
        ctx.close()
        out.append({"left_gb": left_gb, "spp": spp, "free_before_gb": round(free1 / 2**30, 2),
                    "free_after_gb": round(free2 / 2**30, 2), "error": err})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
