#!/usr/bin/env python3
"""Per-launch device time of the wavefront frame against spp, and its fixed cost per launch.

For each spp, one frame runs with MFX_DIAG_ITER=1 (per-iteration HIP events: k_extend / k_camera
and k_shadow of every bounce, the host waiting between iterations) and one without (the frame's
device time as the library enqueues it). A least-squares line t = a + b * spp per launch gives
its fixed cost a. Variants are environment settings, each in its own process:
    launch_sweep.py SCENE SPP[,SPP...] [NAME:VAR=VAL[;VAR=VAL]] ...
e.g. launch_sweep.py scenes/spot.xml 8,16,32,64 default: chunk256:MFX_CHUNK=256
MFX_SWEEP_LIB=path runs a variant library (scripts/build_variant.sh)."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(scene, spps):
    sys.path.insert(0, ROOT)
    if os.environ.get("MFX_SWEEP_LIB"):  # a build_variants/*.so instead of the in-tree library
        import mafrixraytracing_amd.abi as abi
        abi._lib = abi.load_library(os.environ["MFX_SWEEP_LIB"])
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(scene)
    out = {}
    with NativeContext(a, seed=DEFAULT_SEED) as ctx:
        for spp in spps:
            ms = []
            for k in range(3):
                ctx.accum_clear()
                ctx.trace_accumulate(spp, k * spp)
                ctx.sync()
                ms.append(ctx.last_trace_ms())
            c = ctx.ray_counts()
            out[spp] = {"frame_ms": min(ms[1:]), "rays": c[0] + c[1] + c[2]}
    os.environ["MFX_DIAG_ITER"] = "1"
    import tempfile
    tf = tempfile.TemporaryFile()
    saved = os.dup(2)
    sys.stderr.flush()
    os.dup2(tf.fileno(), 2)
    err = None
    try:
        with NativeContext(a, seed=DEFAULT_SEED) as ctx:
            for spp in spps:
                for k in range(2):
                    sys.stderr.write(f"@@ spp {spp} rep {k}\n")
                    sys.stderr.flush()
                    ctx.accum_clear()
                    ctx.trace_accumulate(spp, k * spp)
                    ctx.sync()
    except Exception as e:  # noqa: BLE001 (reported with the captured library output below)
        err = e
    sys.stderr.flush()
    os.dup2(saved, 2)
    tf.seek(0)
    text = tf.read().decode()
    if err is not None:
        print(text[-3000:], file=sys.stderr)
        raise err
    cur = None
    for line in text.splitlines():
        m = re.match(r"@@ spp (\d+) rep (\d+)", line)
        if m:
            cur = (int(m.group(1)), int(m.group(2)))
            if cur[1] == 1:
                out[cur[0]]["launch_ms"] = []
            continue
        m = re.search(r"extend ([\d.]+) ms shadow ([\d.]+) ms", line)
        if m and cur and cur[1] == 1:
            out[cur[0]]["launch_ms"] += [float(m.group(1)), float(m.group(2))]
    print(json.dumps(out))


def fit(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx else 0.0
    return my - b * mx, b


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2], [int(s) for s in sys.argv[3].split(",")])
    scene, spps = sys.argv[1], sys.argv[2]
    variants = sys.argv[3:] or ["default:"]
    for v in variants:
        name, _, envs = v.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(";")):
            k, _, val = kv.partition("=")
            env[k] = val
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", scene, spps], env=env,
                           capture_output=True, text=True, timeout=600)
        if p.returncode:
            print(p.stdout[-2000:], p.stderr[-3000:])
            raise SystemExit(f"variant {name} failed: exit status {p.returncode}")
        d = {int(k): x for k, x in json.loads(p.stdout.strip().splitlines()[-1]).items()}
        xs = sorted(d)
        print(f"=== {name} ({envs or 'defaults'})")
        for s in xs:
            lm = " ".join(f"{t:7.3f}" for t in d[s]["launch_ms"])
            print(f"spp {s:4d}: frame {d[s]['frame_ms']:8.3f} ms {d[s]['rays'] / d[s]['frame_ms'] / 1e3:8.1f} Mrays/s"
                  f" | launches {lm}")
        if len(xs) > 1:
            a, b = fit(xs, [d[s]["frame_ms"] for s in xs])
            print(f"frame: fixed {a:.3f} ms + {b:.4f} ms/spp")
            nl = min(len(d[s]["launch_ms"]) for s in xs)
            fixed = []
            for i in range(nl):
                fa, fb = fit(xs, [d[s]["launch_ms"][i] for s in xs])
                fixed.append(f"{fa:.3f}+{fb:.4f}/spp")
            print("per launch (ext/cam, shadow per bounce):", " ".join(fixed))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
