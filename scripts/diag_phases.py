#!/usr/bin/env python3
"""k_shadow phase shares from a stamp build (-DMFX_DIAG_STAMPS=2) per iteration: the whole frame
traced with MFX_DIAG_ITER=1 and the cumulative stamp counters parsed from its stderr lines
(fetch = list hand-out, scan = window scan, shade = shading batches, node, leaf, fin).
Usage: diag_phases.py LIB.so SCENE SPP"""
import os, re, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = f'''
import sys; sys.path.insert(0, {ROOT!r})
import mafrixraytracing_amd.abi as abi
abi._lib = abi.load_library(sys.argv[1])
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
ctx = NativeContext(load_scene_file(sys.argv[2]), seed=DEFAULT_SEED)
ctx.accum_clear(); ctx.trace_accumulate(int(sys.argv[3]), 0); ctx.sync()
'''
env = dict(os.environ, MFX_DIAG_ITER="1")
p = subprocess.run([sys.executable, "-c", CHILD] + sys.argv[1:4], capture_output=True, text=True, env=env, timeout=300)
prev = None
for line in p.stderr.splitlines():
    m = re.search(r"iter (\d+):.*shadow ([\d.]+) ms; stamps (\S+) (\S+) (\S+) (\S+) outer.*scan (\S+) shade (\S+)", line)
    if not m:
        if "wavefront" in line: print(line)
        continue
    it, ms = int(m.group(1)), float(m.group(2))
    cur = [float(m.group(k)) for k in (3, 4, 5, 6, 7, 8)]  # fetch node leaf fin scan shade (cumulative)
    d = [c - (prev[i] if prev else 0) for i, c in enumerate(cur)]
    prev = cur
    tot = sum(d) or 1
    names = ["handout", "node", "leaf", "fin", "scan", "shade"]
    print(f"iter {it}: k_shadow {ms:.3f} ms; " + ", ".join(f"{n} {v / tot:.3f}" for n, v in zip(names, d)))
if p.returncode:
    print(p.stderr[-2000:])
