#!/usr/bin/env python3
"""Register-spill report of the trace kernels' ISA (gfx950), per kernel instance: VGPRs, scratch
bytes per lane, and the spill code inside loops — scratch loads / stores (VGPR spills) and
v_readlane / v_writelane (SGPR spills to VGPR lanes) — listed by basic block with its loop depth.
Round 4 found bounce-1 k_extend's per-lane ray counter spilled this way: a scratch load-add-store
in every refill. Compiles csrc/mfx_wavefront.hip to assembly on the host (no GPU).
Usage: scripts/isa_spills.py [kernel-name-substring ...]   (default: the flat trace kernels)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mafrixraytracing_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", f"-I{ROOT}/include"]


def compile_asm():
    out = os.path.join(tempfile.mkdtemp(), "wf.s")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "--cuda-device-only", "-S", "-o", out,
                    os.path.join(SRC, "mfx_wavefront.hip")], check=True, capture_output=True)
    return open(out).read()


def kernels(asm):
    for m in re.finditer(r"^(_Z\w+):", asm, re.M):
        name = m.group(1)
        end = asm.index("s_endpgm", m.end())
        meta = re.search(r"; NumVgprs: (\d+)", asm[end:end + 4000])
        scr = re.search(r"; ScratchSize: (\d+)", asm[end:end + 4000])
        yield name, asm[m.end():end], (meta.group(1) if meta else "?"), (scr.group(1) if scr else "?")


def blocks(body):
    cur = ["entry", "", []]
    out = [cur]
    for line in body.split("\n"):
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", line)
        if m:
            cur = [m.group(1), m.group(2), []]
            out.append(cur)
            continue
        t = line.strip()
        if line.startswith("\t") and t and not t.startswith((".", ";")):
            cur[2].append(t.split()[0])
    return out


def main():
    want = sys.argv[1:] or ["k_extendILb0ELb0ELi0ELb0E", "k_extendILb0ELb0ELi0ELb1E", "k_shadowILb0ELb1ELi4ELi0ELb0E",
                            "k_shadowILb0ELb1ELi4ELi0ELb1E", "k_cameraILb0E"]
    asm = compile_asm()
    for name, body, vgpr, scratch in kernels(asm):
        if not any(w in name for w in want):
            continue
        bl = blocks(body)
        ins = sum(len(b[2]) for b in bl)
        rl = sum(b[2].count("v_readlane_b32") for b in bl)
        wl = sum(b[2].count("v_writelane_b32") for b in bl)
        print(f"{name}: {ins} instructions, VGPRs {vgpr}, scratch {scratch} B/lane, v_readlane {rl}, v_writelane {wl}")
        for lab, comment, ops in bl:
            d = re.search(r"Depth=(\d+)", comment)
            if not d:
                continue
            sc = sum(1 for o in ops if o.startswith("scratch_"))
            r = ops.count("v_readlane_b32") + ops.count("v_writelane_b32")
            if sc or r >= 8:
                print(f"  {lab:>12} loop depth {d.group(1)}: {len(ops):4d} instr, scratch ops {sc}, SGPR spill lane ops {r}")


if __name__ == "__main__":
    main()
